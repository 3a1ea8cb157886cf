#!/bin/bash
# Final check of HEAD: GPU suite, smoke, 2-minute randomised soak, default bench
# line, config-5 lines, then kernel traces + FETCH/WRITE of config 5 (pool,
# fresh) and RS(8,14) for the profile index.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 240 python3 -u tools/fuzz_stripes.py --seconds 120 --seed 91 > $O/fuzz.json 2> $O/fuzz.err || exit 3
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 4
C5="--k 64 --n 80 --shard 65536 --stripes 16384"
timeout -k 10 240 python3 bench.py $C5 --cpu-seconds 0 --steps 20 --warmup 3 > $O/cfg5_fresh.json 2>> $O/err.log || exit 5
timeout -k 10 240 python3 bench.py $C5 --cpu-seconds 0 --steps 20 --warmup 3 --pattern-pool 256 > $O/cfg5_pool.json 2>> $O/err.log || exit 6
timeout -k 10 240 python3 bench.py $C5 --cpu-seconds 0 --steps 20 --warmup 3 --mode reconstruct > $O/cfg5_fresh_rec.json 2>> $O/err.log || exit 7
timeout -k 10 240 python3 bench.py $C5 --cpu-seconds 0 --steps 20 --warmup 3 --mode reconstruct --emin 16 --emax 16 > $O/cfg5_e16_rec.json 2>> $O/err.log || exit 8
PROF_TAG=r03ae_cfg5_pool PROF_ARGS="$C5 --pattern-pool 256" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 9
PROF_TAG=r03ae_cfg5_fresh PROF_ARGS="$C5" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 10
PROF_TAG=r03ae_rs8_14 PROF_ARGS="--k 8 --n 14" timeout -k 10 900 bash tools/profile.sh > /dev/null 2>&1 || exit 11
echo done
