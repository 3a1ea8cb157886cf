#!/bin/bash
# Staging device aliases cached per allocation: latency probe x3, then one
# probe run under rocprofv3 (kernel + HIP API trace, no counters) to place
# the single-message calls' kernels and API calls on one timeline.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zero_copy.py tests/test_plugin.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 2; }
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o run --output-format csv -- python3 tools/probe_latency.py --reps 100 > $O/probe_traced.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 3; }
ls -la $O/trace/*
echo done
