#!/bin/bash
# r06v: mailbox jobs' arguments in the kernel arguments (no job board reads):
# mailbox + host-API parity, per-job stamps, config-1 traces and leg.
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mailbox.py tests/test_gpu_parity.py tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_gpu_fuzz_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for W in decode encode; do
  RSMI_PIN_GPU_NUMA=1 RSMI_MAILBOX_STAMPS=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_stamps.trace 2>&1 || { tail $O/${W}_stamps.trace; exit 2; }
  cat $O/${W}_stamps.trace
done
for rep in 1 2 3; do
  for W in decode encode; do
    RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_$rep.trace 2>&1 || { tail $O/${W}_$rep.trace; exit 3; }
  done
done
for f in $O/*_[123].trace; do echo "$f: $(grep -h 'median' $f | grep -v RSMI | sed 's/ over 1000 calls.*//')"; done
for rep in 1 2; do
  timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_$rep.json 2> $O/c1_$rep.err || { tail $O/c1_$rep.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/c1_$rep.json')); print(d['codec']['encode_ms'], d['codec']['decode4_ms'], d['cpu_1t']['avx2_1t'], d['gpu_vs_1core'])"
done
