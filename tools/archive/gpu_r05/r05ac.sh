#!/bin/bash
# The batch-size sweep twice (box-to-box / run-to-run spread of the large batches).
set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_batch_sweep.py --reps 15 > $O/batch_sweep_$r.json 2> $O/batch_sweep_$r.err || { tail -10 $O/batch_sweep_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/batch_sweep_$r.json')); print(d['encode_ms_per_message'], d['decode_ms_per_message'], d['cpu_avx2_1t_encode_ms'], d['cpu_avx2_1t_decode_ms'])"
done
