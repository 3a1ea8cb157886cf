#!/bin/bash
# No completion event between a staged message's chunk kernels
# (RSMI_CHUNK_EVENTS=0: the outputs are copied out after the last chunk) vs
# one event per chunk (default): host-API GPU tests with the variant, then
# the latency probe interleaved, three reps.
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
RSMI_CHUNK_EVENTS=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zero_copy.py tests/test_plugin.py tests/test_gpu_fuzz_host.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_ev1_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 2; }
  RSMI_CHUNK_EVENTS=0 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_ev0_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 3; }
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
echo done
