#!/bin/bash
# Where a config-1 decode's time goes: the latency probe with pinned
# survivors into a pageable dst and 16-byte shards (the fixed cost of a
# call), three reps.
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 2; }
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
echo done
