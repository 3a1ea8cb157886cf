#!/bin/bash
# r02bp: XCD region sweep of the split-table RS(8,14) encode (RSMI_XCD_ENC_REGION, blocks per region; 0 = natural).
set -o pipefail
O=gpurun_out/r02bp
mkdir -p $O
for rep in 1 2; do
  for r in 0 2 8 32 128 1024; do
    echo "== region $r rep $rep" >> $O/sweep.log
    RSMI_XCD_ENC_REGION=$r timeout -k 10 240 python3 bench.py --k 8 --n 14 --cpu-seconds 0 --steps 5 --warmup 2 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], b['reconstruct_ms'])" >> $O/sweep.log 2>> $O/err.log || exit 1
  done
done
echo done
