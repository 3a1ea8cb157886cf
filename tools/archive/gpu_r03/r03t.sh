#!/bin/bash
# Where the config-5 fresh-pattern reconstruct loses against a pool of 256:
# the pool with its pattern sort switched off (RSMI_NO_SORT=1) vs on, and
# fresh patterns both ways (20 steps x 2 reps, reconstruct only).
set -o pipefail
O=gpurun_out/r03t
mkdir -p $O
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 20 --warmup 3 --mode reconstruct"
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 $B $EXTRA 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag', d['value'], b['reconstruct_ms'])" >> $O/ab.log
}
for rep in 1 2; do
  EXTRA="--pattern-pool 256" one "pool sorted" RSMI_X=1 || exit 1
  EXTRA="--pattern-pool 256" one "pool unsorted" RSMI_NO_SORT=1 || exit 2
  EXTRA="" one "fresh sorted" RSMI_X=1 || exit 3
  EXTRA="" one "fresh unsorted" RSMI_NO_SORT=1 || exit 4
  EXTRA="--pattern-pool 4096" one "pool4096 sorted" RSMI_X=1 || exit 5
done
echo done
