#!/bin/bash
# r06o: mailbox grid with a block group per chunk job (the chunks' PCIe reads
# overlap); A/B of the first chunk's share (RSMI_FIRST_CHUNK_PCT) with the
# grid on / off, interleaved; mailbox + host-API parity.
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mailbox.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_mailbox.log 2>&1 || { tail -40 $O/pytest_mailbox.log; exit 1; }
tail -1 $O/pytest_mailbox.log
run() {
  local name=$1; shift
  env "$@" RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_${name}_$rep.trace 2>&1 || { tail $O/${W}_${name}_$rep.trace; exit 2; }
}
for rep in 1 2 3; do
  for W in decode encode; do
    run mb1p50 RSMI_MAILBOX=1
    run mb0p50 RSMI_MAILBOX=0
    run mb1p33 RSMI_MAILBOX=1 RSMI_FIRST_CHUNK_PCT=33
    run mb1p40 RSMI_MAILBOX=1 RSMI_FIRST_CHUNK_PCT=40
    run mb0p33 RSMI_MAILBOX=0 RSMI_FIRST_CHUNK_PCT=33
  done
done
grep -H "median" $O/*.trace | grep -v RSMI | sed 's/ over 1000 calls.*//' | sort
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_gpu_fuzz_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 3; }
tail -1 $O/pytest_host.log
