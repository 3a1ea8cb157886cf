#!/bin/bash
# rs_decode_batch staged survivors read in place over PCIe (chunked,
# non-temporal staging) vs round 4's DMA staging: the decode-batch tests,
# then the config-1 leg's codec figures under both (interleaved).
set -o pipefail
O=gpurun_out/r05n${TAG:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_capi_c.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for dma in 0 1; do
    RSMI_BATCH_DMA=$dma timeout -k 10 200 python3 -c "import json, bench; d = bench.config1_leg(0, 50); print(json.dumps({'dma': $dma, 'codec': d['codec'], 'x': d['gpu_vs_1core']}))" > $O/c1_dma${dma}_$r.json 2> $O/c1_dma${dma}_$r.err || { tail -5 $O/c1_dma${dma}_$r.err; exit 2; }
    cat $O/c1_dma${dma}_$r.json
  done
done
