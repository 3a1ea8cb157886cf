#!/bin/bash
# Fresh-pattern config-5 reconstruct: decode rows stored non-temporally by
# the inversion kernel (lib_ab/invnt) vs the shipped stores (lib_ab/prev),
# 20 steps x 3 reps, reconstruct only and encode + reconstruct.
set -o pipefail
O=gpurun_out/r03y
mkdir -p $O
C5="--k 64 --n 80 --shard 65536 --stripes 16384"
one() {
  local tag=$1 lib=$2; shift 2
  export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so
  timeout -k 10 240 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 3 "$@" 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', d['value'], b['encode_ms'], b['reconstruct_ms'], d['ms_per_step'])" >> $O/ab.log
}
for rep in 1 2 3; do
  for lib in invnt prev; do
    one "fresh-rec" $lib $C5 --mode reconstruct || exit 1
    one "fresh-both" $lib $C5 || exit 2
  done
done
echo done
