#!/bin/bash
# Diagnostics: where a one-stripe device reconstruct's time goes (host call
# time vs HIP events; then a kernel + HIP API trace of the same calls).
set -o pipefail
O=gpurun_out/r04ag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/probe_rec_small.py > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o run --output-format csv -- python3 tools/probe_rec_small.py --reps 50 > $O/probe_traced.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 2; }
echo done
