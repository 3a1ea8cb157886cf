#!/bin/bash
# RS(10,4) reconstruct twin with the pattern inlined in the descriptor
# (membench9 'inline' rows) vs the engine's descriptor -> pattern chain, and
# the default bench line of the current build.
set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 tools/membench9 > $O/membench9.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 2
echo done
