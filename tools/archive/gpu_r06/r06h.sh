#!/bin/bash
# r06h: kernel timeline of config-1 single-message decode / encode calls
# (rocprofv3 kernel trace + HIP runtime API trace, no counters).
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for w in decode encode; do
  timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace -d $GRAFT_REPO_ROOT/$O/$w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/trace_single.py $w 300 > $GRAFT_REPO_ROOT/$O/$w.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
find $O -name "*.csv" | head
