#!/bin/bash
# rs_encode_batch (send-side batching): the new tests first, then the whole
# GPU suite, then the default line (config1 leg: encode_batch64).
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_encode_batch.py tests/test_plugin.py -x -v --timeout 240 --timeout-method thread > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $O/pytest_new.log; exit 1; }
tail -3 $O/pytest_new.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['config1']['codec']), json.dumps(d['config1']['gpu_vs_1core']))"
