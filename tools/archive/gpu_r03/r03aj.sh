#!/bin/bash
# Last check of the committed tree, as the driver runs it: GPU suite, smoke, default bench line.
set -o pipefail
O=gpurun_out/r03aj
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
