#!/bin/bash
# Small batches chunked per message / single-message batches on the single
# path: the whole GPU suite, then the batch-size sweep.
set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/bench_batch_sweep.py --reps 15 > $O/batch_sweep.json 2> $O/batch_sweep.err || { tail -10 $O/batch_sweep.err; exit 2; }
cat $O/batch_sweep.json
