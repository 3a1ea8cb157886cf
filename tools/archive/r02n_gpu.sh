# r02n: copy-pool width A/B on the staged host paths (8 vs 16 workers),
# and SQ counters of the BLAKE2b kernel (65,536 x 1 KiB and 256 x 1 MiB).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02n
mkdir -p $O
for t in 8 16 8 16; do
  RSMI_COPY_THREADS=$t timeout -k 10 300 python3 $R/tools/bench_host_api.py --batch-only --batch-reps 5 > $O/host_api_t${t}_$(date +%s%N).json 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES --kernel-trace -d $O/b2_sq -o run --output-format csv -- python3 $R/tools/bench_blake2b.py --reps 3 > $O/b2_sq.log 2>&1 || exit 2
echo ok
