#!/bin/bash
# r02v: rec kernel duration with a pool of 256 patterns vs a fresh pattern
# per stripe (same box, kernel trace), config 5.
set -euo pipefail
O=gpurun_out/r02v
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pool -o run --output-format csv -- python3 $B --pattern-pool 256 > $O/pool.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fresh -o run --output-format csv -- python3 $B > $O/fresh.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pool_e8 -o run --output-format csv -- python3 $B --pattern-pool 256 --emin 8 --emax 8 > $O/pool_e8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fresh_e8 -o run --output-format csv -- python3 $B --emin 8 --emax 8 > $O/fresh_e8.log 2>&1
echo done
