#!/bin/bash
# r02as: XCD region of the split-table RS(10,4) reconstruct
# (RSMI_XCD_REC_REGION: 0 natural ... 256 = a stripe per XCD), three
# erasure cases, reconstruct only, interleaved.
set -o pipefail
O=gpurun_out/r02as
mkdir -p $O
run() { timeout -k 10 300 python3 bench.py --cpu-seconds 0 --mode reconstruct --steps 8 --warmup 2 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['reconstruct_ms'])"; }
for rep in 1 2; do
  for r in 0 16 64 128 256; do
    export RSMI_XCD_REC_REGION=$r
    echo "== region=$r rep $rep random" >> $O/ab.log; run >> $O/ab.log 2>> $O/ab.err || exit 1
    echo "== region=$r rep $rep one" >> $O/ab.log; run --erase 3 >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== region=$r rep $rep parity" >> $O/ab.log; run --erase 10,11,12,13 >> $O/ab.log 2>> $O/ab.err || exit 3
  done
done
echo ok
