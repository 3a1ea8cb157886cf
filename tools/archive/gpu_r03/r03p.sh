#!/bin/bash
# The N > 1 gather leg rehearsed on one GPU (gloo): a normal run (the line
# carries gather.status ok, verified stripes, no mismatch) and one whose
# watchdog fires (--gather-timeout 1: the line is still printed, exit 0).
set -o pipefail
O=gpurun_out/r03p
mkdir -p $O
RSMI_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --stripes 1000 --steps 3 --warmup 1 --cpu-seconds 2 > $O/gpus2_gather.json 2> $O/gpus2_gather.err || exit 1
RSMI_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --stripes 1000 --steps 3 --warmup 1 --cpu-seconds 0 --gather-timeout 1 > $O/gpus2_watchdog.json 2> $O/gpus2_watchdog.err || exit 2
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/gpus1.json 2> $O/gpus1.err || exit 3
echo done
