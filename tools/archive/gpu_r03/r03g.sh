#!/bin/bash
# Re-entry check of the restored tree: GPU suite, smoke, then r03f (sharded
# N=2 gloo rehearsal, default line, RS(10,4) reconstruct movement twin).
set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
bash tools/gpu/r03f.sh || exit 3
echo done
