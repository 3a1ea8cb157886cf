#!/bin/bash
# r06d: the tree with device sets, the aliasing fixes and the -W/-L syndrome
# kernel: the whole GPU suite, smoke() and the default line (with the new
# device_set leg).
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['breakdown']['reconstruct_GBps'], json.dumps(d['config1']['gpu_vs_1core']), d['config5']['reconstruct'], d['config3_worst']['reconstruct']['frac']); print(json.dumps(d['device_set']))"
