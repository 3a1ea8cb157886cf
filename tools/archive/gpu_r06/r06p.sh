#!/bin/bash
# r06p: first-chunk share 25 / 33 %, write-combined input staging
# (RSMI_STAGE_WC=1), the grid for one-launch arena decodes
# (RSMI_MAILBOX_MIN_JOBS=1), interleaved; the config-1 leg alone.
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_${name}_$rep.trace 2>&1 || { tail $O/${W}_${name}_$rep.trace; exit 2; }
}
for rep in 1 2 3; do
  for W in decode encode; do
    run p33 RSMI_FIRST_CHUNK_PCT=33
    run p25 RSMI_FIRST_CHUNK_PCT=25
    run p33wc RSMI_STAGE_WC=1
  done
done
grep -H "median" $O/*.trace | grep -v RSMI | sed 's/ over 1000 calls.*//' | sort
RSMI_STAGE_WC=1 RSMI_MAILBOX_MIN_JOBS=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_mailbox.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_minjobs1.log 2>&1 || { tail -40 $O/pytest_minjobs1.log; exit 3; }
tail -1 $O/pytest_minjobs1.log
for rep in 1 2; do
  timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_default_$rep.json 2> $O/c1_default_$rep.err || { tail $O/c1_default_$rep.err; exit 4; }
  RSMI_MAILBOX_MIN_JOBS=1 timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_minjobs1_$rep.json 2> $O/c1_minjobs1_$rep.err || { tail $O/c1_minjobs1_$rep.err; exit 4; }
  RSMI_STAGE_WC=1 timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_wc_$rep.json 2> $O/c1_wc_$rep.err || { tail $O/c1_wc_$rep.err; exit 4; }
done
for f in $O/c1_*.json; do echo $f; cat $f; done
