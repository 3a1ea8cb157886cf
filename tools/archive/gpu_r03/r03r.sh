#!/bin/bash
# Solve tables read one parity row ahead (gen_bitslice default now; -s = the
# previous form, lib_ab/prev = HEAD before the change): GPU suite, smoke,
# interleaved config-5 reconstruct A/B (20 steps x 3 reps).
set -o pipefail
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
C5="--k 64 --n 80 --shard 65536 --stripes 16384"
one() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 240 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 3 "$@" 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', d['value'], b['encode_ms'], b['reconstruct_ms'])" >> $O/ab.log
}
for rep in 1 2 3; do
  for lib in cur prev; do
    one "c5-fresh-1..16" $lib $C5 --mode reconstruct || exit 3
    one "c5-pool256" $lib $C5 --mode reconstruct --pattern-pool 256 || exit 4
    one "c5-e16" $lib $C5 --mode reconstruct --emin 16 --emax 16 || exit 5
    one "c5-1..8" $lib $C5 --mode reconstruct --emax 8 || exit 6
    one "rs8_14" $lib --k 8 --n 14 --mode reconstruct || exit 7
  done
done
echo done
