#!/bin/bash
# rocprofv3 evidence of HEAD: for the headline, config 5
# (pool of 256 and a fresh pattern per stripe) and RS(8,14), one kernel-trace
# pass plus separate FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh), then a
# SQ-counter pass of the config-5 fresh reconstruct (tools/pmc_valu.sh).
set -o pipefail
export TMPDIR=/tmp
C5="--k 64 --n 80 --shard 65536 --stripes 16384"
PROF_TAG=r03d_head PROF_ARGS="" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 1
PROF_TAG=r03d_cfg5_pool PROF_ARGS="$C5 --pattern-pool 256" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 2
PROF_TAG=r03d_cfg5_fresh PROF_ARGS="$C5" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 3
PROF_TAG=r03d_rs8_14 PROF_ARGS="--k 8 --n 14" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 4
PMC_TAG=r03d_cfg5_fresh_rec BENCH_ARGS="$C5 --mode reconstruct" timeout -k 10 300 bash tools/pmc_valu.sh > /dev/null 2>&1 || exit 5
echo done
