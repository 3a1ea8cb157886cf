#!/bin/bash
# r02aa: build stream at the lowest priority vs default (config-5 fresh).
set -euo pipefail
O=gpurun_out/r02aa
mkdir -p $O
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 8 --warmup 2"
for rep in 1 2; do
  for pr in default low; do
    RSMI_BUILD_PRIORITY=$pr timeout -k 10 240 $B > $O/both_${pr}_$rep.json 2>> $O/err.log
    RSMI_BUILD_PRIORITY=$pr timeout -k 10 240 $B --mode reconstruct > $O/rec_${pr}_$rep.json 2>> $O/err.log
  done
done
echo done
