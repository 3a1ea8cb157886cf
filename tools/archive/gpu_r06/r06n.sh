#!/bin/bash
# r06n: small-transfer PCIe reads; config-1 single-message A/B on one box:
# mailbox grid on / off, fused present copy (RSMI_FUSED_PRESENT=1), four
# column chunks (RSMI_STAGE_CHUNKS=4), interleaved processes; the fused copy's
# parity under the host-API tests and the fuzzer.
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench/build/pcie_rates > $O/pcie_rates.txt 2>&1 || { cat $O/pcie_rates.txt; exit 1; }
cat $O/pcie_rates.txt
run() {  # name env... -- what
  local name=$1; shift
  env "$@" RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_${name}_$rep.trace 2>&1 || { tail $O/${W}_${name}_$rep.trace; exit 2; }
}
for rep in 1 2 3; do
  W=decode
  run mb1 RSMI_MAILBOX=1
  run mb0 RSMI_MAILBOX=0
  run mb1f RSMI_MAILBOX=1 RSMI_FUSED_PRESENT=1
  run mb0f RSMI_MAILBOX=0 RSMI_FUSED_PRESENT=1
  run mb1c4 RSMI_MAILBOX=1 RSMI_STAGE_CHUNKS=4
  run mb1fc4 RSMI_MAILBOX=1 RSMI_FUSED_PRESENT=1 RSMI_STAGE_CHUNKS=4
  W=encode
  run mb1 RSMI_MAILBOX=1
  run mb0 RSMI_MAILBOX=0
  run mb1c4 RSMI_MAILBOX=1 RSMI_STAGE_CHUNKS=4
done
grep -H "median" $O/*.trace | grep -v RSMI | sed 's/ over 1000 calls.*//' | sort
RSMI_FUSED_PRESENT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_gpu_mailbox.py tests/test_gpu_concurrency.py -m gpu -x -q -k "decode or Decode or mailbox or concurr" --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 3; }
tail -1 $O/pytest_fused.log
RSMI_FUSED_PRESENT=1 timeout -k 10 100 python3 tools/fuzz_host_api.py --seconds 60 --seed 37 > $O/fuzz_fused.json 2> $O/fuzz.err || { tail $O/fuzz.err; cat $O/fuzz_fused.json; exit 4; }
cat $O/fuzz_fused.json
