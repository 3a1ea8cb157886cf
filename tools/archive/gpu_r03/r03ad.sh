#!/bin/bash
# Output ids prefetched into a VGPR in the syndrome kernel's prologue (read by
# readlane in the solve instead of scalar loads per output group) and the slot
# scan moved after the first data loads: the -M diagnostic build over the
# bit-sliced tests (no mask disagreement), the GPU suite, then an interleaved
# A/B against HEAD (lib_ab/prev), 20 steps x 3 reps.
set -o pipefail
O=gpurun_out/r03ad
mkdir -p $O
RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/dbg/librsmi.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -s -m gpu --timeout 120 --timeout-method thread -k "bitslice or xcd or ptrs" > $O/dbg_tests.txt 2>&1 || exit 1
if grep -q RSMI_MASK_MISMATCH $O/dbg_tests.txt; then echo "mask mismatch"; exit 2; fi
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 3
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 240 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 3 "$@" 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', d['value'], b['reconstruct_ms'])" >> $O/ab.log
}
for rep in 1 2 3; do
  for lib in cur prev; do
    one "fresh" $lib $C5 || exit 4
    one "pool256" $lib $C5 --pattern-pool 256 || exit 5
    one "e16" $lib $C5 --emin 16 --emax 16 || exit 6
    one "rs8_14" $lib --k 8 --n 14 --mode reconstruct || exit 7
  done
done
echo done
