set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r01
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_fetch.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_write.log 2>&1 || exit 3
echo done
