#!/bin/bash
# r06z: the arena (in-place) single decode: one launch (default) vs its
# message in column chunks through the mailbox grid (RSMI_INPLACE_CHUNKS=1)
# vs one chunk through the grid (RSMI_MAILBOX_MIN_JOBS=1); interleaved
# config-1 legs; zero-copy parity under both knobs.
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
export TMPDIR=/tmp
RSMI_INPLACE_CHUNKS=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_parity.py -m gpu -x -q -k "zero or arena or pinned or place or alias" --timeout 200 --timeout-method thread > $O/pytest_chunks.log 2>&1 || { tail -30 $O/pytest_chunks.log; exit 1; }
tail -1 $O/pytest_chunks.log
RSMI_MAILBOX_MIN_JOBS=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zero_copy.py tests/test_gpu_parity.py -m gpu -x -q -k "zero or arena or pinned or place or alias" --timeout 200 --timeout-method thread > $O/pytest_min1.log 2>&1 || { tail -30 $O/pytest_min1.log; exit 1; }
tail -1 $O/pytest_min1.log
for rep in 1 2 3; do
  for v in base chunks min1; do
    case $v in base) E="";; chunks) E="RSMI_INPLACE_CHUNKS=1";; min1) E="RSMI_MAILBOX_MIN_JOBS=1";; esac
    env $E timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_${v}_$rep.json 2> $O/c1_${v}_$rep.err || { tail $O/c1_${v}_$rep.err; exit 3; }
    echo "$v $rep $(python3 -c "import json; d=json.load(open('$O/c1_${v}_$rep.json')); c=d['codec']; print(c['decode4_arena_ms'], c['decode4_ms'], c['encode_ms'], d['cpu_1t']['avx2_1t'], d['gpu_vs_1core'])")"
  done
done
