#!/bin/bash
# r06j: the round-6 tree's default bench line and the rocprofv3 passes of
# that same default command (kernel trace, then FETCH_SIZE and WRITE_SIZE in
# runs of their own), summarised per role by tools/prof_line.py, which also
# writes profiles/traffic.json (bench.py's roofline.traffic / traffic_source).
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/line_trace.json 2> $O/line_trace.err || exit 4
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv -- python3 bench.py > $O/line_fetch.json 2> $O/line_fetch.err || exit 5
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv -- python3 bench.py > $O/line_write.json 2> $O/line_write.err || exit 6
python3 tools/prof_line.py $O $O/line_summary.md --bench-json $O/line_trace.json --traffic-json $O/traffic.json --profile profiles/r06j_line_rocprof_summary.md
echo done
