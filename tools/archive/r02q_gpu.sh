#!/bin/bash
# r02q: pattern-cache host cost A/B (growth without a device sync,
# allocation-free pattern creation) and the config-5 reconstruct-only step.
set -euo pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02q
mkdir -p $O
for lib in noise-erasurecode-plugin_amd/lib_ab/r02o/librsmi.so noise-erasurecode-plugin_amd/lib/librsmi.so; do
  tag=$(basename $(dirname $lib))
  RSMI_LIB=$R/$lib timeout -k 10 180 python3 tools/bench_patterns.py > $O/patterns_$tag.json 2>> $O/err.log
  RSMI_LIB=$R/$lib timeout -k 10 240 python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 6 --warmup 2 > $O/cfg5_rec_fresh_$tag.json 2>> $O/err.log
done
echo done
