#!/bin/bash
# SQ counters of the final build's config-5 kernels (fresh 1-16 mix, and 16
# erasures), plus the instruction-cache pass, each in a run of its own.
set -o pipefail
O=gpurun_out/r04ac
mkdir -p $O
export TMPDIR=/tmp
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --cpu-seconds 0 --no-extra-legs --steps 2 --warmup 1"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -d $O/fresh/sq -o run --output-format csv -- python3 bench.py $C5 > $O/fresh.log 2>&1 || { tail -5 $O/fresh.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -d $O/e16/sq -o run --output-format csv -- python3 bench.py $C5 --mode reconstruct --emin 16 --emax 16 > $O/e16.log 2>&1 || { tail -5 $O/e16.log; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace -d $O/fresh/sqc -o run --output-format csv -- python3 bench.py $C5 > $O/sqc.log 2>&1 || { tail -5 $O/sqc.log; exit 3; }
python3 tools/sq_summary.py $O/fresh $O/e16 > $O/sq_summary.md 2>&1 || { cat $O/sq_summary.md; exit 4; }
cat $O/sq_summary.md
echo done
