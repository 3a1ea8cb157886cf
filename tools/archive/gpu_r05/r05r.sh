#!/bin/bash
# Batched calls bounded by the pinned-staging cap: the batch, plugin, zero-copy
# and C-harness GPU tests.
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_encode_batch.py tests/test_plugin.py tests/test_gpu_zero_copy.py tests/test_capi_c.py tests/test_gpu_concurrency.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
