#!/bin/bash
# The GPU suite after the RSMI_SMALL_SPLIT=0 fix (the knob now really keeps
# small calls on the syndrome kernel; rs_stat counts the stripes each kernel
# reconstructed and the tests assert which one ran), then the randomised
# fuzzers on the round-5 engine: device stripes (every code, small and large
# calls, both small-call routings) and the host API.
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 tools/fuzz_stripes.py --seconds 150 --seed 5 > $O/fuzz_stripes.json 2> $O/fuzz_stripes.err || { tail -5 $O/fuzz_stripes.err; exit 2; }
cat $O/fuzz_stripes.json
timeout -k 10 200 python3 tools/fuzz_host_api.py --seconds 150 --seed 5 > $O/fuzz_host.json 2> $O/fuzz_host.err || { tail -5 $O/fuzz_host.err; exit 3; }
cat $O/fuzz_host.json
echo done
