#!/bin/bash
# r02p: config-5 reconstruct time vs erasure count (fresh patterns), the
# syndrome kernel vs the split-table kernel (RSMI_BITSLICE_REC_MIN_E).
set -euo pipefail
O=gpurun_out/r02p
mkdir -p $O
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 6 --warmup 2"
for e in 1 2 3 4 6 8 12 16; do
  timeout -k 10 240 $B --emin $e --emax $e > $O/syn_e$e.json 2>> $O/err.log
done
for e in 1 2 3 4 6; do
  RSMI_BITSLICE_REC_MIN_E=99 timeout -k 10 240 $B --emin $e --emax $e > $O/split_e$e.json 2>> $O/err.log
done
timeout -k 10 240 $B > $O/syn_mix.json 2>> $O/err.log
timeout -k 10 240 $B --pattern-pool 256 > $O/syn_mix_pool.json 2>> $O/err.log
echo done
