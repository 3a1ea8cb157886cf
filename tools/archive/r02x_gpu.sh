#!/bin/bash
# r02x: config-1 host-API latency, and its HIP-operation breakdown.
set -euo pipefail
O=gpurun_out/r02x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/bench_decode_latency.py > $O/latency.json 2> $O/err.log
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bench_decode_latency.py --reps 100 > $O/trace.log 2>&1
echo done
