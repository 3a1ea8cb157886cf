#!/bin/bash
# r02ak: XCD-aware block order (xcd.hpp) -- GPU suite, then RSMI_XCD=0/1
# interleaved on the headline and the config-5 shapes (mode both).
# AB_X lists the settings ("0 1"; "def" = unset: the per-kernel default);
# AB_TAG names the output directory.
set -o pipefail
O=gpurun_out/${AB_TAG:-r02ak}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
run() { timeout -k 10 300 python3 bench.py --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], b['reconstruct_ms'], d['roofline']['frac'])"; }
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --steps 10 --warmup 3"
for rep in 1 2; do
  for x in ${AB_X:-0 1}; do
    if [ $x = def ]; then unset RSMI_XCD; else export RSMI_XCD=$x; fi
    echo "== xcd=$x rep $rep: headline" >> $O/ab.log; run >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== xcd=$x rep $rep: cfg5 pool 256" >> $O/ab.log; run $C5 --pattern-pool 256 >> $O/ab.log 2>> $O/ab.err || exit 3
    echo "== xcd=$x rep $rep: cfg5 fresh" >> $O/ab.log; run $C5 >> $O/ab.log 2>> $O/ab.err || exit 4
    echo "== xcd=$x rep $rep: cfg5 e=16" >> $O/ab.log; run $C5 --emin 16 --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 5
    echo "== xcd=$x rep $rep: rs8_14" >> $O/ab.log; run --k 8 --n 14 >> $O/ab.log 2>> $O/ab.err || exit 6
  done
done
echo ok
