#!/bin/bash
# Concurrency soaks on the final build: 8 threads on one context for 120 s
# each -- RS(64,16) with a small pattern cap (evictions while other threads
# read the cache), and RS(10,4) with config-1-sized messages (host-API calls
# on the two-chunk staged path, decode batches, device-stripe reconstructs).
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
export TMPDIR=/tmp
RSMI_PATTERN_CAP=2000 timeout -k 10 200 python3 -u tools/soak_concurrency.py --seconds 120 --threads 8 > $O/soak_64_80.json 2> $O/soak_64_80.err || { echo "soak 64:80 failed"; cat $O/soak_64_80.json; tail -20 $O/soak_64_80.err; exit 1; }
cat $O/soak_64_80.json
timeout -k 10 200 python3 -u tools/soak_concurrency.py --seconds 120 --threads 8 --code 10:14 --shard 104858 > $O/soak_10_14.json 2> $O/soak_10_14.err || { echo "soak 10:14 failed"; cat $O/soak_10_14.json; tail -20 $O/soak_10_14.err; exit 2; }
cat $O/soak_10_14.json
echo done
