#!/bin/bash
# membench11: can a clock-phased read/write schedule (the whole chip reading
# in one window and writing in the next, s_memrealtime as the reference)
# raise the RS(10,4) encode shape's movement rate above the mixed stream's?
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 240 ./tools/membench11 > $O/mb11.log 2>&1 || { cat $O/mb11.log; exit 1; }
cat $O/mb11.log
