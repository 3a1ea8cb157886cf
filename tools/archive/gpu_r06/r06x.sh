#!/bin/bash
# r06x: batched host calls in 4 / 6 / 8 message chunks (RSMI_BATCH_CHUNKS),
# interleaved config-1 legs; mailbox tests with the gave-up flag; batch
# parity with 8 chunks.
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mailbox.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_mailbox.log 2>&1 || { tail -30 $O/pytest_mailbox.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_mailbox.log | tail -14
RSMI_BATCH_CHUNKS=8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encode_batch.py tests/test_gpu_zero_copy.py tests/test_gpu_fuzz_host.py tests/test_plugin.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_b8.log 2>&1 || { tail -30 $O/pytest_b8.log; exit 2; }
tail -1 $O/pytest_b8.log
for rep in 1 2; do
  for bc in 4 8 6; do
    RSMI_BATCH_CHUNKS=$bc timeout -k 10 300 python3 tools/config1_leg.py 100 > $O/c1_b${bc}_$rep.json 2> $O/c1_b${bc}_$rep.err || { tail $O/c1_b${bc}_$rep.err; exit 3; }
    echo "b$bc $rep $(python3 -c "import json; d=json.load(open('$O/c1_b${bc}_$rep.json')); c=d['codec']; print(c['decode4_batch64_ms_per_message'], c['encode_batch64_ms_per_message'], d['gpu_vs_1core'])")"
  done
done
for bc in 4 8; do
  RSMI_BATCH_CHUNKS=$bc RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py decode_batch 400 > $O/decode_batch_b$bc.trace 2>&1 || exit 4
  RSMI_BATCH_CHUNKS=$bc RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py encode_batch 400 > $O/encode_batch_b$bc.trace 2>&1 || exit 4
done
head -3 $O/*_batch_b*.trace
