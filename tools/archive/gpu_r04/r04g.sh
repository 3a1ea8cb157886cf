#!/bin/bash
# Single-message in-place decode (engine-pinned survivors read where they
# are) + the GPU suite; latency probe; host API table.
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || exit 2
done
cat $O/probe_*.json
timeout -k 10 300 python3 tools/bench_host_api.py --reps 30 > $O/host_api.json 2> $O/host_api.err || exit 3
cat $O/host_api.json
echo done
