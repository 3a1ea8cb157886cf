#!/bin/bash
# Headline RS(10,4): pattern-sorted reconstruct descriptors (shipped) vs
# address order (RSMI_NO_SORT=1), interleaved, 20 steps x 3 reps.
set -o pipefail
O=gpurun_out/r03v
mkdir -p $O
for rep in 1 2 3; do
  for ns in 0 1; do
    if [ $ns = 1 ]; then export RSMI_NO_SORT=1; else unset RSMI_NO_SORT; fi
    timeout -k 10 240 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 3 2>> $O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('nosort=$ns', d['value'], b['encode_ms'], b['reconstruct_ms'])" >> $O/ab.log || exit 1
  done
done
echo done
