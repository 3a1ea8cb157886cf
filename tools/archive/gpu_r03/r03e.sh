#!/bin/bash
# Config-5 reconstruct A/B of the row-subset syndrome kernels
# (RSMI_BITSLICE_TOPS=0 vs default, interleaved; fresh patterns and a pool of
# 256), the 16-erasure control, and a same-box A/B of the variants' prefetch
# depth (lib_ab/q3: t8 at 4 waves/SIMD).
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 10 --warmup 3 --mode reconstruct"
for rep in 1 2; do
  for tops in 1 0; do
    RSMI_BITSLICE_TOPS=$tops timeout -k 10 240 $B > $O/fresh_tops${tops}_$rep.json 2>> $O/err.log || exit 4
    RSMI_BITSLICE_TOPS=$tops timeout -k 10 240 $B --pattern-pool 256 > $O/pool_tops${tops}_$rep.json 2>> $O/err.log || exit 5
  done
done
timeout -k 10 240 $B --emin 16 --emax 16 > $O/e16.json 2>> $O/err.log || exit 6
AB_TAG=r03e/ab AB_LIBS="cur q3" AB_REPS=2 timeout -k 10 600 bash tools/ab_libs.sh > /dev/null 2>&1 || exit 7
echo done
