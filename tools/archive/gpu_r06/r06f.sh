#!/bin/bash
# r06f: host copy rates on the box and the single-message phase medians.
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 60 tools/ubench/build/stage_copy > $O/stage_copy.log 2>&1 || exit 1
for w in decode encode; do
  RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 1000 > $O/$w.trace 2>&1 || exit 2
done
lscpu | grep -i "model name\|flags" | cut -c1-300 > $O/lscpu.txt
cat $O/stage_copy.log $O/*.trace
