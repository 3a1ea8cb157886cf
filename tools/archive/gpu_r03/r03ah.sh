#!/bin/bash
# Config-3 erasure cases on HEAD (reconstruct only, 6,553 stripes x 1 MiB):
# random 1-4, one data shard, 4 data shards (0-3 and 6-9), 4 parity shards;
# and config 2's second mode (streamed from pinned host memory).
set -o pipefail
O=gpurun_out/r03ah
mkdir -p $O
B="python3 bench.py --cpu-seconds 0 --steps 10 --warmup 3 --mode reconstruct"
timeout -k 10 240 $B > $O/rand14.json 2>> $O/err.log || exit 1
timeout -k 10 240 $B --erase 3 > $O/one_data.json 2>> $O/err.log || exit 2
timeout -k 10 240 $B --erase 0,1,2,3 > $O/data0123.json 2>> $O/err.log || exit 3
timeout -k 10 240 $B --erase 6,7,8,9 > $O/data6789.json 2>> $O/err.log || exit 4
timeout -k 10 240 $B --erase 10,11,12,13 > $O/parity4.json 2>> $O/err.log || exit 5
timeout -k 10 300 python3 bench.py --stream --cpu-seconds 0 --steps 3 --warmup 1 > $O/stream.json 2>> $O/err.log || exit 6
echo done
