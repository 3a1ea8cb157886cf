#!/bin/bash
# r02br: bit-sliced RS(8,14) shipped by default: GPU suite, smoke, RS(8,14) and default lines, kernel trace of RS(8,14).
set -o pipefail
O=gpurun_out/r02br
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 240 python3 bench.py --k 8 --n 14 --cpu-seconds 0 > $O/rs8_14_$rep.json 2>> $O/err.log || exit 3
  RSMI_BITSLICE=0 timeout -k 10 240 python3 bench.py --k 8 --n 14 --cpu-seconds 0 > $O/rs8_14_split_$rep.json 2>> $O/err.log || exit 4
done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o rs8_14 -- python3 bench.py --k 8 --n 14 --cpu-seconds 0 --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 6
echo done
