#!/bin/bash
# Check of HEAD after the row-guard default change: GPU suite, smoke, a 2-minute
# randomised soak, the default bench line and config 5 (fresh, pool).
set -o pipefail
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 240 python3 -u tools/fuzz_stripes.py --seconds 120 --seed 77 > $O/fuzz.json 2> $O/fuzz.err || exit 3
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 4
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 20 --warmup 3"
timeout -k 10 240 python3 bench.py $C5 > $O/cfg5_fresh.json 2>> $O/err.log || exit 5
timeout -k 10 240 python3 bench.py $C5 --pattern-pool 256 > $O/cfg5_pool.json 2>> $O/err.log || exit 6
timeout -k 10 240 python3 bench.py $C5 --mode reconstruct > $O/cfg5_fresh_rec.json 2>> $O/err.log || exit 7
echo done
