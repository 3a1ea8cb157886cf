#!/bin/bash
# Final build (bit-plane transposes with v_bitop3 selects): GPU suite, smoke, default bench line,
# config-5 lines (pool, fresh, 16 erasures), RS(8,14), config 2 streamed.
set -o pipefail
O=gpurun_out/r02final3
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --steps 10 --warmup 3"
timeout -k 10 240 $B --pattern-pool 256 > $O/cfg5_pool.json 2>> $O/err.log || exit 4
timeout -k 10 240 $B > $O/cfg5_fresh.json 2>> $O/err.log || exit 5
timeout -k 10 240 $B --emin 16 --emax 16 > $O/cfg5_e16.json 2>> $O/err.log || exit 6
timeout -k 10 240 python3 bench.py --k 8 --n 14 --cpu-seconds 0 > $O/rs8_14.json 2>> $O/err.log || exit 7
timeout -k 10 240 python3 bench.py --stream --steps 3 --warmup 1 > $O/stream.json 2>> $O/err.log || exit 8
echo done
