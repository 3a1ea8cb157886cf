#!/bin/bash
# r06i: a single message's second column chunk on its own stream vs one stream.
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
for rep in 1 2; do
for mode in 2 1; do
  for w in decode encode; do
    RSMI_CHUNK_STREAMS=$mode RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 1000 > $O/${w}_streams${mode}_$rep.trace 2>&1 || exit 2
  done
done
done
timeout -k 10 600 python3 -u -m pytest tests/test_plugin.py tests/test_gpu_parity.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_gpu_fuzz_host.py tests/test_capi_c.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
grep -H "median" $O/*.trace | grep -v RSMI
cat $O/decode_streams2_1.trace
