#!/bin/bash
# After the arena batches moved to the direct form: the decode-batch and C
# harness tests, the config-1 codec figures (direct vs DMA), then both
# randomised fuzzers (the host-API one now with encode/decode batches).
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_gpu_concurrency.py tests/test_capi_c.py tests/test_gpu_encode_batch.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for dma in 0 1; do
  RSMI_BATCH_DMA=$dma timeout -k 10 200 python3 -c "import json, bench; d = bench.config1_leg(0, 50); print(json.dumps({'dma': $dma, 'codec': d['codec'], 'x': d['gpu_vs_1core']}))" > $O/c1_dma${dma}.json 2> $O/c1_dma${dma}.err || { tail -5 $O/c1_dma${dma}.err; exit 2; }
  cat $O/c1_dma${dma}.json
done
timeout -k 10 200 python3 tools/fuzz_host_api.py --seconds 120 --seed 6 > $O/fuzz_host.json 2> $O/fuzz_host.err || { tail -5 $O/fuzz_host.err; cat $O/fuzz_host.json; exit 3; }
cat $O/fuzz_host.json
timeout -k 10 200 python3 tools/fuzz_stripes.py --seconds 100 --seed 6 > $O/fuzz_stripes.json 2> $O/fuzz_stripes.err || { tail -5 $O/fuzz_stripes.err; exit 4; }
cat $O/fuzz_stripes.json
