#!/bin/bash
# r02bq: bit-sliced RS(8,14) (lib_ab/b814: BITSLICE_CODES += 8:14) vs the split-table kernels;
# movement twin with the RS(8,14) shape (tools/membench8).
set -o pipefail
O=gpurun_out/r02bq
mkdir -p $O
L=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/b814/librsmi.so
RSMI_LIB=$L RSMI_BITSLICE=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "not kernel_selection and not row_group_of_six" --timeout 240 --timeout-method thread > $O/tests_b814_forced.txt 2>&1 || exit 1
run() { timeout -k 10 240 python3 bench.py --k 8 --n 14 --cpu-seconds 0 --steps 5 --warmup 2 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], b['reconstruct_ms'])"; }
for rep in 1 2; do
  echo "== split (shipped) rep $rep" >> $O/ab.log; run >> $O/ab.log 2>> $O/err.log || exit 2
  echo "== bitslice enc + syndrome rec rep $rep" >> $O/ab.log; RSMI_LIB=$L RSMI_BITSLICE=1 run >> $O/ab.log 2>> $O/err.log || exit 3
  echo "== bitslice enc + split rec rep $rep" >> $O/ab.log; RSMI_LIB=$L RSMI_BITSLICE=1 RSMI_BITSLICE_REC=0 run >> $O/ab.log 2>> $O/err.log || exit 4
done
echo done
