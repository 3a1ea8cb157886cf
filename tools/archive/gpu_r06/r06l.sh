#!/bin/bash
# r06l: a single message's chunk-0 event (the marker between the two kernels)
# on / off, interleaved processes, plus the r06k checks.
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
for mode in 1 0; do
  for w in decode encode; do
    RSMI_CHUNK_EVENTS=$mode RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 1000 > $O/${w}_ev${mode}_$rep.trace 2>&1 || exit 2
  done
done
done
for w in encode_batch decode_batch; do
  RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $w 400 > $O/$w.trace 2>&1 || exit 5
done
grep -H "median" $O/*.trace | grep -v RSMI
cat $O/encode_batch.trace $O/decode_batch.trace
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_device_set.py tests/test_gpu_fuzz_host.py tests/test_capi_c.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RSMI_CHUNK_EVENTS=0 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_plugin.py -m gpu -x -q -k "decode or encode" --timeout 300 --timeout-method thread > $O/pytest_ev0.log 2>&1 || { tail -30 $O/pytest_ev0.log; exit 3; }
tail -1 $O/pytest_ev0.log
timeout -k 10 240 python3 tools/fuzz_host_api.py --seconds 150 --seed 29 > $O/fuzz.json 2> $O/fuzz.err || { tail $O/fuzz.err; cat $O/fuzz.json; exit 4; }
cat $O/fuzz.json
