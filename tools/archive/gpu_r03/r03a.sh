#!/bin/bash
# Round-3 entry check: GPU suite + smoke, the default line, bench.py --gpus 2
# self-launching two ranks (gloo rehearsal on one GPU), and the HIP API trace
# of lease-buffer growth.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
RSMI_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --stripes 3000 --steps 5 --warmup 2 --cpu-seconds 4 > $O/gpus2_gloo.json 2> $O/gpus2_gloo.err || exit 4
timeout -k 10 300 rocprofv3 --hip-trace --stats -d $O/growth -o run --output-format csv -- python3 tools/growth_trace.py > $O/growth.json 2> $O/growth.err || exit 5
echo done
