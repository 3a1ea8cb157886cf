#!/bin/bash
# GPU suite (rollback, growth, hash policy, row-subset syndrome kernels,
# chunked gather), smoke, and the hash-policy crossover sweep.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 tools/bench_hash_policy.py > $O/hash_policy.json 2> $O/hash_policy.err || exit 3
echo done
