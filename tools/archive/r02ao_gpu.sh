#!/bin/bash
# r02ao: stripes per XCD region for the bit-sliced RS(64,16) kernels
# (RSMI_XCD_BS_STRIPES), config 5 mode both, interleaved.
set -o pipefail
O=gpurun_out/r02ao
mkdir -p $O
RSMI_XCD_BS_STRIPES=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "bitslice or wide_code" --timeout 120 --timeout-method thread > $O/tests_bs4.txt 2>&1 || exit 1
run() { timeout -k 10 300 python3 bench.py --cpu-seconds 0 --k 64 --n 80 --shard 65536 --stripes 16384 --steps 10 --warmup 3 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], b['reconstruct_ms'])"; }
for rep in 1 2; do
  for r in 1 2 4 8; do
    echo "== stripes/region=$r rep $rep fresh" >> $O/ab.log; RSMI_XCD_BS_STRIPES=$r run >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== stripes/region=$r rep $rep pool" >> $O/ab.log; RSMI_XCD_BS_STRIPES=$r run --pattern-pool 256 >> $O/ab.log 2>> $O/ab.err || exit 3
  done
done
echo ok
