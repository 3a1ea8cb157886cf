#!/bin/bash
# Kernel trace of the RS(64,16) latency sweep at 16,384 and 1,024 stripes:
# separates kernel time from host time in the per-call latency.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bench_latency_sweep.py --k 64 --n 80 --shard 65536 --batches 1024,16384 --reps 5 > $O/sweep.json 2> $O/sweep.err || exit 1
echo done
