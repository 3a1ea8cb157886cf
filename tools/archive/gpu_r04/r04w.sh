#!/bin/bash
# Host-API fuzz on the final build: the seeded GPU test, then 150 s of random
# cases (tools/fuzz_host_api.py) and 120 s of the device-stripe fuzz
# (tools/fuzz_stripes.py) with fresh seeds.
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fuzz_host.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python3 -u tools/fuzz_host_api.py --seconds 150 --seed 4242 > $O/fuzz_host.json 2> $O/fuzz_host.err || { echo "fuzz_host failed"; cat $O/fuzz_host.json; tail -20 $O/fuzz_host.err; exit 2; }
cat $O/fuzz_host.json
timeout -k 10 220 python3 -u tools/fuzz_stripes.py --seconds 120 --seed 4243 > $O/fuzz_stripes.json 2> $O/fuzz_stripes.err || { echo "fuzz_stripes failed"; cat $O/fuzz_stripes.json; tail -20 $O/fuzz_stripes.err; exit 3; }
cat $O/fuzz_stripes.json
echo done
