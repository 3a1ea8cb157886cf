#!/bin/bash
# Round-4 build: GPU suite; config-1 latency breakdown with the polled
# completion wait (RSMI_SYNC_SPIN_US) and the copy-pool spin; the default
# bench line (the driver's command) and its kernel trace.
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || exit 2
  RSMI_SYNC_SPIN_US=0 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_nosync_$rep.json 2>> $O/probe.err || exit 3
  RSMI_COPY_SPIN_US=50 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_spin50_$rep.json 2>> $O/probe.err || exit 4
done
cat $O/probe_*.json
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 5
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 1 > $O/bench_trace.json 2> $O/bench_trace.err || exit 6
echo done
