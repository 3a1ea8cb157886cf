#!/bin/bash
# Staged column chunks per small message (RSMI_STAGE_CHUNKS 1-4) on the
# round-5 engine (non-temporal staging): config-1 pageable encode / decode.
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for ch in 2 3 4 1; do
    RSMI_STAGE_CHUNKS=$ch timeout -k 10 150 python3 tools/probe_latency.py --reps 300 > $O/lat_ch${ch}_$r.json 2> $O/lat_ch${ch}_$r.err || { tail -5 $O/lat_ch${ch}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/lat_ch${ch}_$r.json')); print('chunks $ch rep $r', d['encode_pageable'], d['decode_pageable'], d['cpu_avx2_encode'])"
  done
done
