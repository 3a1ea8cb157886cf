#!/bin/bash
# r06m: the mailbox grid for single staged messages (MailboxCall): its tests,
# config-1 encode / decode per-call phases with the grid on / off
# (interleaved processes), the host-API parity suites through it, a fuzz
# run and a full bench line.
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mailbox.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_mailbox.log 2>&1 || { tail -40 $O/pytest_mailbox.log; exit 1; }
tail -1 $O/pytest_mailbox.log
for rep in 1 2; do
for mode in 1 0; do
  for w in decode encode; do
    RSMI_MAILBOX=$mode RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 1000 > $O/${w}_mb${mode}_$rep.trace 2>&1 || { tail $O/${w}_mb${mode}_$rep.trace; exit 2; }
  done
done
done
grep -H "median" $O/*.trace | grep -v RSMI
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_gpu_fuzz_host.py tests/test_gpu_encode_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 3; }
tail -1 $O/pytest_host.log
timeout -k 10 150 python3 tools/fuzz_host_api.py --seconds 90 --seed 31 > $O/fuzz.json 2> $O/fuzz.err || { tail $O/fuzz.err; cat $O/fuzz.json; exit 4; }
cat $O/fuzz.json
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
cat $O/bench.json
