#!/bin/bash
# r06a: device-set contexts and the dst-aliasing fixes on the GPU.
set -o pipefail
mkdir -p gpurun_out/r06a
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_device_set.py tests/test_gpu_zero_copy.py tests/test_capi_c.py \
  "tests/test_gpu_parity.py::test_decode_dst_overlapping_survivors" -m gpu \
  > gpurun_out/r06a/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r06a/pytest.log
exit $rc
