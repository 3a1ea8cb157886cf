#!/bin/bash
# Latency per stripe batch: RS(64,16) 64 KiB shards and
# the headline RS(10,4) 1 MiB shards, 1 .. 16,384 / 6,553 stripes.
set -o pipefail
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_latency_sweep.py --k 64 --n 80 --shard 65536 > $O/latency_rs64_16.json 2> $O/latency_rs64_16.err || exit 1
timeout -k 10 300 python3 -u tools/bench_latency_sweep.py --k 10 --n 14 --shard 1048576 --batches 1,2,4,8,16,32,64,128,256,512,1024,2048,4096,6553 > $O/latency_rs10_4.json 2> $O/latency_rs10_4.err || exit 2
echo done
