#!/bin/bash
# SQ counters of the current syndrome reconstruct (every stripe in the full
# kernel, mask-record prologue): fresh 1..16 mix, pool of 256, e = 1..4 and
# e = 16; plus the sharded placement under torchrun world 1 over RCCL
# (sharded_run after the refactor).
set -o pipefail
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct"
PMC_TAG=r03q_fresh BENCH_ARGS="$C5" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 1
PMC_TAG=r03q_pool BENCH_ARGS="$C5 --pattern-pool 256" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 2
PMC_TAG=r03q_e4 BENCH_ARGS="$C5 --emax 4" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 3
PMC_TAG=r03q_e16 BENCH_ARGS="$C5 --emin 16 --emax 16" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 4
PMC_TAG=r03q_enc BENCH_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --mode encode" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 5
mkdir -p gpurun_out/r03q
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 1 --placement sharded --stripes 1000 --steps 3 --warmup 1 > gpurun_out/r03q/sharded_rccl_w1.json 2> gpurun_out/r03q/sharded_rccl_w1.err || exit 6
echo done
