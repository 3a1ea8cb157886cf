#!/bin/bash
# The tree with both batch forms direct: GPU suite, smoke(), the default
# line, and the concurrency soaks (every host-API entry point incl.
# rs_encode_batch) on RS(64,16) with evictions and on config-1-sized RS(10,4).
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['config1']['gpu_vs_1core']))"
RSMI_PATTERN_CAP=2000 timeout -k 10 120 python3 tools/soak_concurrency.py --seconds 40 --threads 8 > $O/soak64.json 2> $O/soak64.err || { tail -5 $O/soak64.err; exit 4; }
cat $O/soak64.json
timeout -k 10 120 python3 tools/soak_concurrency.py --seconds 40 --threads 8 --code 10:14 --shard 104858 > $O/soak10.json 2> $O/soak10.err || { tail -5 $O/soak10.err; exit 5; }
cat $O/soak10.json
