#!/bin/bash
# Round-4 starting point on the round-3 build: config-1 host-API latency
# (rs_encode / rs_decode of the 1,048,580-B blob, pageable and pinned) and
# the config-5 line (RS(64,16), 64 KiB shards, fresh 1-16 patterns) with a
# kernel trace.
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 300 python3 tools/bench_host_api.py --reps 50 > $O/host_api.json 2> $O/host_api.err &&
timeout -k 10 200 python3 bench.py --cpu-seconds 0 --steps 5 --warmup 2 --k 64 --n 80 --shard 65536 --stripes 16384 > $O/cfg5.json 2> $O/cfg5.err &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/cfg5_trace -o run -- python3 bench.py --cpu-seconds 0 --steps 5 --warmup 2 --k 64 --n 80 --shard 65536 --stripes 16384 > $O/cfg5_prof.json 2> $O/cfg5_prof.err
echo "rc=$?"
