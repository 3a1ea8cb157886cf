#!/bin/bash
# Latency per stripe batch on the final build:
# RS(64,16) with 64 KiB shards and RS(10,4) with 1 MiB shards.
set -o pipefail
O=gpurun_out/r04ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_latency_sweep.py --k 64 --n 80 --shard 65536 > $O/sweep_64_80.json 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep_64_80.json
timeout -k 10 300 python3 tools/bench_latency_sweep.py --k 10 --n 14 --shard 1048576 > $O/sweep_10_14.json 2>> $O/sweep.err || { tail -20 $O/sweep.err; exit 2; }
cat $O/sweep_10_14.json
echo done
