#!/bin/bash
# After the mask-record prologue: a 5-minute randomised soak of every kernel
# family (tools/fuzz_stripes.py), then config-5 kernel traces + FETCH/WRITE
# passes of the current build (pool of 256 and fresh patterns).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 400 python3 -u tools/fuzz_stripes.py --seconds 300 --seed 31 > $O/fuzz.json 2> $O/fuzz.err || exit 1
C5="--k 64 --n 80 --shard 65536 --stripes 16384"
PROF_TAG=r03o_cfg5_pool PROF_ARGS="$C5 --pattern-pool 256" timeout -k 10 600 bash tools/profile.sh > /dev/null 2>&1 || exit 2
PROF_TAG=r03o_cfg5_fresh PROF_ARGS="$C5" timeout -k 10 600 bash tools/profile.sh > /dev/null 2>&1 || exit 3
echo done
