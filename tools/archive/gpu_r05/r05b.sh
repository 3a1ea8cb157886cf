#!/bin/bash
# membench10: one-factor decomposition of the config-5 reconstruct's movement
# shape (fresh 1-16, 1-4, 16 erasures); membench9 (RS(10,4) reconstruct twin)
# on the same box.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 120 ./tools/membench10 16384 1 16 > $O/mb10_fresh.log 2>&1 || { cat $O/mb10_fresh.log; exit 1; }
timeout -k 10 120 ./tools/membench10 16384 1 4 > $O/mb10_e1_4.log 2>&1 || exit 2
timeout -k 10 120 ./tools/membench10 16384 16 16 > $O/mb10_e16.log 2>&1 || exit 3
timeout -k 10 120 ./tools/membench9 > $O/mb9.log 2>&1 || exit 4
cat $O/*.log
