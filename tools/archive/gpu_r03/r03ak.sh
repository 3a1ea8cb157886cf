#!/bin/bash
# The N > 1 line with its gather leg rehearsed at N = 4 on one GPU (gloo).
set -o pipefail
O=gpurun_out/r03ak
mkdir -p $O
RSMI_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 4 --stripes 1000 --steps 3 --warmup 1 --cpu-seconds 2 --gather-stripes 256 > $O/gpus4_gather.json 2> $O/gpus4_gather.err || exit 1
echo done
