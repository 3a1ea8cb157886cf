#!/bin/bash
# bench.py with the configs[2] worst-case leg: its GPU test, then the default line.
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['config3_worst']), json.dumps(d['config1']['gpu_vs_1core']))"
