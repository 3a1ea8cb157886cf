#!/bin/bash
# r06s: the full GPU suite on the new defaults (mailbox grid, three chunks
# 25/35/40 %); config-1 leg with the caller held on one CPU (default) or
# node-wide, interleaved; write-combined staging under the new split; the
# default bench line.
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_cpu_$rep.json 2> $O/c1_cpu_$rep.err || { tail $O/c1_cpu_$rep.err; exit 2; }
  cat $O/c1_cpu_$rep.json
  RSMI_C1_PIN=node timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_node_$rep.json 2> $O/c1_node_$rep.err || { tail $O/c1_node_$rep.err; exit 2; }
  cat $O/c1_node_$rep.json
  RSMI_STAGE_WC=1 timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_wc_$rep.json 2> $O/c1_wc_$rep.err || { tail $O/c1_wc_$rep.err; exit 2; }
  cat $O/c1_wc_$rep.json
done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
cat $O/bench.json
