#!/bin/bash
# Row-subset syndrome kernels without row guards (gen_bitslice default now;
# lib_ab/guard = the guarded build, -u): GPU suite, same-box A/B on the
# config-5 reconstruct shapes (+ lib_ab/t12: -T 4,8,12), RSMI_BITSLICE_TOPS=0 control, SQ counters.
set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
AB_TAG=r03h/ab AB_LIBS="cur guard t12" AB_REPS=2 timeout -k 10 900 bash tools/ab_libs.sh > /dev/null 2>&1 || exit 2
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 10 --warmup 3"
for rep in 1 2; do
  for tops in 1 0; do
    RSMI_BITSLICE_TOPS=$tops timeout -k 10 240 $B --mode reconstruct > $O/fresh_tops${tops}_$rep.json 2>> $O/err.log || exit 4
    RSMI_BITSLICE_TOPS=$tops timeout -k 10 240 $B --mode reconstruct --pattern-pool 256 > $O/pool_tops${tops}_$rep.json 2>> $O/err.log || exit 5
  done
done
timeout -k 10 240 $B > $O/cfg5_both_fresh.json 2>> $O/err.log || exit 6
timeout -k 10 240 $B --pattern-pool 256 > $O/cfg5_both_pool.json 2>> $O/err.log || exit 7
PMC_TAG=r03h_cfg5_fresh_rec BENCH_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 8
echo done
