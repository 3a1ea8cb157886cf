#!/bin/bash
# r02bs: headline RS(10,4) with the generated bit-sliced kernels forced (RSMI_BITSLICE=1) vs the shipped split-table kernels.
set -o pipefail
O=gpurun_out/r02bs
mkdir -p $O
run() { timeout -k 10 300 python3 bench.py --cpu-seconds 0 --steps 10 --warmup 3 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], b['reconstruct_ms'])"; }
for rep in 1 2; do
  echo "== split (shipped) rep $rep" >> $O/ab.log; run >> $O/ab.log 2>> $O/err.log || exit 1
  echo "== bitslice enc + syndrome rec rep $rep" >> $O/ab.log; RSMI_BITSLICE=1 run >> $O/ab.log 2>> $O/err.log || exit 2
  echo "== bitslice enc + split rec rep $rep" >> $O/ab.log; RSMI_BITSLICE=1 RSMI_BITSLICE_REC=0 run >> $O/ab.log 2>> $O/err.log || exit 3
done
echo done
