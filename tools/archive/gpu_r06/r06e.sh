#!/bin/bash
# r06e: where a config-1 message's rs_decode / rs_encode time goes (RSMI_TRACE phases).
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
for w in decode encode; do
  timeout -k 10 120 python3 tools/trace_single.py $w 400 > $O/$w.plain 2>&1 || exit 1
  RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 400 > $O/$w.trace 2>&1 || exit 2
done
tail -n 30 $O/*.plain $O/*.trace
