#!/bin/bash
# Column-chunked staging of small host-API messages (the second half staged
# while the kernel codes the first): GPU suite, then the latency probe with
# 1 / 2 (default for >= 256 KiB) / 3 chunks.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for nch in 1 2 3; do
    RSMI_STAGE_CHUNKS=$nch timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_c${nch}_$rep.json 2>> $O/probe.err || exit 2
  done
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
echo done
