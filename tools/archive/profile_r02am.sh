# r02am profiles after the XCD-aware block order: headline RS(10,4) and
# config 5 RS(64,16) 64 KiB shards (pool of 256 patterns), kernel trace +
# FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh), plus the default bench line.
set -o pipefail
mkdir -p gpurun_out/r02am
timeout -k 10 400 python3 bench.py > gpurun_out/r02am/bench.json 2> gpurun_out/r02am/bench.err || exit 1
PROF_TAG=r02am bash tools/profile.sh || exit 2
PROF_TAG=r02am_cfg5 PROF_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256" bash tools/profile.sh || exit 3
