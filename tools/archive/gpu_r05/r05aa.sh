#!/bin/bash
# Per-message cost of rs_encode_batch / rs_decode_batch against batch size
# (config-1 messages, pageable), with one AVX2 core as the yardstick.
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_batch_sweep.py --reps 15 > $O/batch_sweep.json 2> $O/batch_sweep.err || { tail -10 $O/batch_sweep.err; exit 1; }
cat $O/batch_sweep.json
