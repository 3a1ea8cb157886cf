#!/bin/bash
# Pattern builds ordered after the caller's queued work (no overlap with the
# previous kernels; RSMI_BUILD_OVERLAP=1 restores it) + one-wave inversion
# workgroups: GPU suite, smoke, interleaved A/B against HEAD (lib_ab/prev).
set -o pipefail
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
C5="--k 64 --n 80 --shard 65536 --stripes 16384"
one() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 240 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 3 "$@" 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', d['value'], b['encode_ms'], b['reconstruct_ms'], d['ms_per_step'])" >> $O/ab.log
}
for rep in 1 2 3; do
  for lib in cur prev; do
    one "c5-fresh-rec" $lib $C5 --mode reconstruct || exit 3
    one "c5-fresh-both" $lib $C5 || exit 4
    one "c5-pool-both" $lib $C5 --pattern-pool 256 || exit 5
    one "c5-e16-rec" $lib $C5 --mode reconstruct --emin 16 --emax 16 || exit 6
    one "headline" $lib || exit 7
  done
done
echo done
