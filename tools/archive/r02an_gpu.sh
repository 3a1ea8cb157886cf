#!/bin/bash
# r02an: XCD regions for the split-table RS(10,4) encode (RSMI_XCD_ENC_REGION
# = blocks per region; 0 natural, 256 = a stripe per XCD).  GPU suite with the
# default build and with region 8 forced (bijection check), then encode-only
# timings interleaved.
set -o pipefail
O=gpurun_out/r02an
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
RSMI_XCD_ENC_REGION=8 timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_region8.txt 2>&1 || exit 2
run() { timeout -k 10 300 python3 bench.py --cpu-seconds 0 --mode encode "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], d['roofline']['frac'])"; }
for rep in 1 2; do
  for r in 0 1 2 4 8 32 256; do
    echo "== region=$r rep $rep" >> $O/ab.log; RSMI_XCD_ENC_REGION=$r run >> $O/ab.log 2>> $O/ab.err || exit 3
  done
done
echo ok
