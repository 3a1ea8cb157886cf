#!/bin/bash
# r02u: pattern builds on a context-owned build stream (overlapping queued
# kernels) -- A/B vs the r02s build; concurrency/eviction/parity tests.
set -euo pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 8 --warmup 2"
for rep in 1 2; do
for lib in noise-erasurecode-plugin_amd/lib_ab/r02s/librsmi.so noise-erasurecode-plugin_amd/lib/librsmi.so; do
  tag=$(basename $(dirname $lib))
  RSMI_LIB=$R/$lib timeout -k 10 240 $B > $O/fresh_both_${tag}_$rep.json 2>> $O/err.log
  RSMI_LIB=$R/$lib timeout -k 10 240 $B --mode reconstruct > $O/fresh_rec_${tag}_$rep.json 2>> $O/err.log
done
done
echo done
