#!/bin/bash
# Non-temporal staging copies (rsmi::stage_copy) vs memcpy on the config-1
# host-API path: tools/probe_latency.py, interleaved reps.
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for nt in 1 0; do
    RSMI_STAGE_NT=$nt timeout -k 10 150 python3 tools/probe_latency.py --reps 400 > $O/lat_nt${nt}_$r.json 2> $O/lat_nt${nt}_$r.err || { tail -5 $O/lat_nt${nt}_$r.err; exit 1; }
    echo "nt=$nt rep $r"; cat $O/lat_nt${nt}_$r.json
  done
done
