#!/bin/bash
# The sharded placement rehearsed at N=2 (gloo, one GPU), the default line,
# and the RS(10,4) reconstruct movement twin (tools/membench9.hip).
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
RSMI_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --placement sharded --stripes 1500 --steps 3 --warmup 1 > $O/sharded2_gloo.json 2> $O/sharded2_gloo.err || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 300 tools/membench9 > $O/membench9.log 2>&1 || exit 3
echo done
