#!/bin/bash
# r02r: pattern cache with GPU-derived rows, flat index, radix stripe sort,
# no device sync on table growth: GPU suite, pattern host-cost A/B,
# config-5 reconstruct-only (fresh patterns), headline bench.
set -euo pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
for lib in noise-erasurecode-plugin_amd/lib_ab/r02o/librsmi.so noise-erasurecode-plugin_amd/lib/librsmi.so; do
  tag=$(basename $(dirname $lib))
  RSMI_LIB=$R/$lib timeout -k 10 180 python3 tools/bench_patterns.py > $O/patterns_$tag.json 2>> $O/err.log
  RSMI_LIB=$R/$lib timeout -k 10 240 python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 6 --warmup 2 > $O/cfg5_rec_fresh_$tag.json 2>> $O/err.log
done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2>> $O/err.log
echo done
