#!/bin/bash
# r06k: device-set tests (member ownership), the host-API fuzzer with the
# aliasing cases (pytest seeds + a 150-s run).
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_device_set.py tests/test_gpu_fuzz_host.py tests/test_capi_c.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python3 tools/fuzz_host_api.py --seconds 150 --seed 29 > $O/fuzz.json 2> $O/fuzz.err || { tail $O/fuzz.err; cat $O/fuzz.json; exit 2; }
cat $O/fuzz.json
