#!/bin/bash
# r02w: why fresh patterns slow the syndrome kernel: instruction-fetch and
# stall counters, pool vs fresh (one rocprofv3 --pmc pass each).
set -uo pipefail
O=gpurun_out/r02w
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -i "SQC_ICACHE\|SQ_IFETCH\|SQ_INST_CYCLES\|SQ_WAIT_INST\|SQC_TC_INST" $O/counters.txt | head -40 > $O/counters_icache.txt || true
B="bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 3 --warmup 1"
for mode in pool fresh; do
  extra=""; [ $mode = pool ] && extra="--pattern-pool 256"
  timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --kernel-trace -d $O/${mode}_sq -o run --output-format csv -- python3 $B $extra > $O/${mode}_sq.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES --kernel-trace -d $O/${mode}_sqc -o run --output-format csv -- python3 $B $extra > $O/${mode}_sqc.log 2>&1 || echo "sqc pass failed for $mode"
done
echo done
