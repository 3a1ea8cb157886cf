#!/bin/bash
# Syndrome-kernel prologue from the host's per-descriptor mask record
# (bitslice.hpp BsStripeMask): GPU suite, then a same-box interleaved A/B
# against the previous build (lib_ab/prev), 20 steps x 3 reps.
set -o pipefail
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
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
    one "c5-1..4" $lib $C5 --mode reconstruct --emax 4 || exit 6
    one "rs8_14" $lib --k 8 --n 14 --mode reconstruct || exit 7
  done
done
echo done
