#!/bin/bash
# GPU suite (rollback, growth, hash policy, row-subset syndrome kernels,
# chunked gather), the hash-policy crossover sweep, config-5 reconstruct A/B
# of the row-subset kernels (RSMI_BITSLICE_TOPS=0 vs default, interleaved),
# the sharded placement rehearsed at N=2 (gloo), and the default line.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 tools/bench_hash_policy.py > $O/hash_policy.json 2> $O/hash_policy.err || exit 3
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 10 --warmup 3 --mode reconstruct"
for rep in 1 2; do
  for tops in 1 0; do
    RSMI_BITSLICE_TOPS=$tops timeout -k 10 240 $B > $O/fresh_tops${tops}_$rep.json 2>> $O/err.log || exit 4
    RSMI_BITSLICE_TOPS=$tops timeout -k 10 240 $B --pattern-pool 256 > $O/pool_tops${tops}_$rep.json 2>> $O/err.log || exit 5
  done
done
timeout -k 10 240 $B --emin 16 --emax 16 > $O/e16.json 2>> $O/err.log || exit 6
RSMI_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --placement sharded --stripes 1500 --steps 3 --warmup 1 > $O/sharded2_gloo.json 2> $O/sharded2_gloo.err || exit 7
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 8
timeout -k 10 300 tools/membench9 > $O/membench9.log 2>&1 || exit 9
echo done
