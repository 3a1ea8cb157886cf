#!/bin/bash
# Small-message copies split over the copy pool: the staged path's copies
# (staging, present shares, outputs) now go through CopyPool::run, which
# stays inline under 2 x RSMI_COPY_PART_MIN (default 1 MiB: inline for every
# staged message).  GPU suite with parts of 128 KiB and spinning workers, then
# the latency probe: default / parts 128 KiB / parts 256 KiB, workers spinning
# 300 us, two reps each.
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
RSMI_COPY_PART_MIN=131072 RSMI_COPY_SPIN_US=300 timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_split.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_def_$rep.json 2>> $O/probe.err || exit 2
  RSMI_COPY_PART_MIN=131072 RSMI_COPY_SPIN_US=300 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_p128_$rep.json 2>> $O/probe.err || exit 3
  RSMI_COPY_PART_MIN=262144 RSMI_COPY_SPIN_US=300 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_p256_$rep.json 2>> $O/probe.err || exit 4
  RSMI_COPY_PART_MIN=131072 RSMI_COPY_SPIN_US=300 RSMI_COPY_THREADS=3 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_p128t3_$rep.json 2>> $O/probe.err || exit 5
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
echo done
