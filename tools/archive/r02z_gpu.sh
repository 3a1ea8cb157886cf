#!/bin/bash
# r02z: invert_patterns_kernel with 64 vs 256 threads per pattern.
set -euo pipefail
O=gpurun_out/r02z
mkdir -p $O
export TMPDIR=/tmp
for t in 64 256; do
  RSMI_INVERT_THREADS=$t timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_$t.txt 2>&1
  RSMI_INVERT_THREADS=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 tools/bench_patterns.py > $O/patterns_$t.json 2> $O/prof_$t.log
  RSMI_INVERT_THREADS=$t timeout -k 10 240 python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 8 --warmup 2 > $O/fresh_both_$t.json 2>> $O/err.log
  RSMI_INVERT_THREADS=$t timeout -k 10 240 python3 bench.py --k 10 --n 14 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 4 --warmup 1 --mode reconstruct > $O/rs10_4_$t.json 2>> $O/err.log
done
echo done
