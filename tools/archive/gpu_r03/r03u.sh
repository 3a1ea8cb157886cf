#!/bin/bash
# Concurrency soak of the round-3 build (mask records, builds ordered after
# the caller's stream, one-wave inversion): 8 threads, pattern cap 2,000.
set -o pipefail
O=gpurun_out/r03u
mkdir -p $O
RSMI_PATTERN_CAP=2000 timeout -k 10 240 python3 -u tools/soak_concurrency.py --seconds 150 --threads 8 > $O/soak.json 2> $O/soak.err || exit 1
echo done
