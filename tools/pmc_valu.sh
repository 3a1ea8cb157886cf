# PMC passes on one bench configuration (BENCH_ARGS): wave/VALU/wait
# cycles and instruction-cache behaviour of the coding kernels.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_${PMC_TAG:-valu}
mkdir -p $O
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY SQ_IFETCH SQ_WAVES --kernel-trace -d $O/sq -o run --output-format csv -- $B > $O/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace -d $O/sqc -o run --output-format csv -- $B > $O/sqc.log 2>&1 || exit 2
echo done
