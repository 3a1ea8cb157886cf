#!/bin/bash
# r02y: host-pipeline chunk size for small calls (config-1 message) A/B:
# quarter-of-the-call chunks (>= 256 KiB) vs one 8 MiB-class chunk.
set -euo pipefail
O=gpurun_out/r02y
mkdir -p $O
for rep in 1 2; do
  RSMI_CHUNK_BYTES=8388608 timeout -k 10 120 python3 tools/bench_decode_latency.py > $O/lat_8m_$rep.json 2>> $O/err.log
  timeout -k 10 120 python3 tools/bench_decode_latency.py > $O/lat_auto_$rep.json 2>> $O/err.log
  RSMI_CHUNK_BYTES=131072 timeout -k 10 120 python3 tools/bench_decode_latency.py > $O/lat_128k_$rep.json 2>> $O/err.log
done
timeout -k 10 300 python3 tools/bench_host_api.py > $O/host_api.json 2>> $O/err.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
echo done
