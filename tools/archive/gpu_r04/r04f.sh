#!/bin/bash
# Config-1 latency after the copy-pool change (jobs under 2 MiB copied inline
# on the caller), the receive-batching numbers (bench_host_api), and the
# rocprof passes of the default bench line: kernel trace + FETCH_SIZE +
# WRITE_SIZE (separate runs), summarised by tools/prof_line.py.
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || exit 2
done
cat $O/probe_*.json
timeout -k 10 300 python3 tools/bench_host_api.py --reps 30 > $O/host_api.json 2> $O/host_api.err || exit 3
cat $O/host_api.json
P="python3 bench.py --steps 5 --warmup 2 --cpu-seconds 1 --config1-reps 20 --config5-steps 3 --config5-warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $P > $O/line_trace.json 2> $O/line_trace.err || exit 4
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv -- $P > $O/line_fetch.json 2> $O/line_fetch.err || exit 5
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv -- $P > $O/line_write.json 2> $O/line_write.err || exit 6
python3 tools/prof_line.py $O $O/line_summary.md --bench-json $O/line_trace.json
echo done
