#!/bin/bash
# r02t: config-5 lines (mode both) after the pattern-cache rework: pool of
# 256 patterns, a fresh pattern per stripe, 16 erasures per stripe; RS(8,14).
set -euo pipefail
O=gpurun_out/r02t
mkdir -p $O
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 10 --warmup 3"
timeout -k 10 240 $B --pattern-pool 256 > $O/cfg5_pool.json 2>> $O/err.log
timeout -k 10 240 $B > $O/cfg5_fresh.json 2>> $O/err.log
timeout -k 10 240 $B --emin 16 --emax 16 > $O/cfg5_e16.json 2>> $O/err.log
timeout -k 10 240 python3 bench.py --k 8 --n 14 --cpu-seconds 0 > $O/rs8_14.json 2>> $O/err.log
echo done
