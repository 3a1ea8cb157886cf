#!/bin/bash
# r06g: single-message calls with the helper's async copies vs all on the caller.
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
for rep in 1 2; do
for mode in 1 0; do
  for w in decode encode; do
    RSMI_ASYNC_COPIES=$mode RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 1000 > $O/${w}_async${mode}_$rep.trace 2>&1 || exit 2
  done
done
done
timeout -k 10 600 python3 -u -m pytest tests/test_plugin.py tests/test_gpu_parity.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_gpu_fuzz_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
grep -H "median" $O/*.trace
cat $O/decode_async1_1.trace $O/encode_async1_1.trace
