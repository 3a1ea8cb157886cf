#!/bin/bash
# Hash policy: GPU tests of the crossover and prepareShards overlap, then the
# host/GPU crossover sweep (tools/bench_hash_policy.py).
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_blake2b.py tests/test_plugin.py tests/test_gpu_concurrency.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 600 python3 tools/bench_hash_policy.py > $O/hash_policy.json 2> $O/hash_policy.err || exit 2
echo done
