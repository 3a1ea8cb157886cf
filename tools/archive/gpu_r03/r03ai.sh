#!/bin/bash
# Syndrome reconstruct prefetch depth 5 and 6 inputs (BITSLICE_REC_PREFETCH, lib_ab/p5, p6) vs 4 (HEAD).
set -o pipefail
O=gpurun_out/r03ai
mkdir -p $O
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 240 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 3 "$@" 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', d['value'], b['reconstruct_ms'])" >> $O/ab.log
}
for rep in 1 2 3; do
  for lib in cur p5 p6; do
    one "e16" $lib $C5 --emin 16 --emax 16 || exit 1
    one "pool256" $lib $C5 --pattern-pool 256 || exit 2
    one "fresh" $lib $C5 || exit 3
    one "rs8_14" $lib --k 8 --n 14 --mode reconstruct || exit 4
  done
done
echo done
