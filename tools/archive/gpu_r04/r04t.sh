#!/bin/bash
# Odd column chunks of a staged message on the lease's second stream (chunk
# kernels no longer serialise behind each other's end-of-kernel and event):
# host-API GPU tests, then the latency probe with RSMI_STAGE_STREAMS=1 (one
# stream) and the default (two), interleaved, three reps.
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zero_copy.py tests/test_plugin.py tests/test_capi_c.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  RSMI_STAGE_STREAMS=1 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_s1_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 2; }
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_s2_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 3; }
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
echo done
