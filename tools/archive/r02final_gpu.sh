#!/bin/bash
# End of round 2: GPU suite, smoke, default bench line, headline and
# config-5 profiles (kernel trace + FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02final
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
PROF_TAG=r02final bash tools/profile.sh || exit 4
PROF_TAG=r02final_cfg5 PROF_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256" bash tools/profile.sh || exit 5
echo done
