#!/bin/bash
# Longer interleaved A/B (20 steps, 3 reps) of the config-5 reconstruct:
# full syndrome kernel only (RSMI_BITSLICE_TOPS=0), row-subset t4/t8 (shipped
# build) and t4/t8/t12 (lib_ab/t12).
set -o pipefail
O=gpurun_out/r03i
mkdir -p $O
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 20 --warmup 3 --mode reconstruct"
one() {  # tag, env..., then bench args after --
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 240 $B "$@" 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag', d['value'], b['reconstruct_ms'], b['reconstruct_kernel'])" >> $O/ab.log
}
T12=RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/t12/librsmi.so
for rep in 1 2 3; do
  for shape in "e1-4:--emax 4" "e1-16:--emax 16" "pool:--emax 16 --pattern-pool 256" "e1-8:--emax 8"; do
    name=${shape%%:*}; args=${shape#*:}
    one "$name tops0" RSMI_BITSLICE_TOPS=0 -- $args || exit 2
    one "$name t4,8" RSMI_BITSLICE_TOPS=1 -- $args || exit 3
    one "$name t4,8,12" $T12 -- $args || exit 4
  done
done
echo done
