# r02f: config-5 reconstruct A/B (current vs round-1 build): bench lines and
# rocprofv3 kernel stats of each, to split host-side from kernel time.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${R02F_TAG:-r02f}
mkdir -p $O
A="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --steps 5 --warmup 2 --cpu-seconds 0"
for rep in 1; do
  for lib in cur r01; do
    if [ $lib = r01 ]; then export RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/r01/librsmi.so; else unset RSMI_LIB; fi
    timeout -k 10 300 python3 $R/bench.py $A > $O/bench_${lib}_${rep}.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 $R/bench.py $A --pattern-pool 256 > $O/bench_pool_${lib}_${rep}.json 2>> $O/err.log || exit 2
  done
done
for lib in cur r01; do
  if [ $lib = r01 ]; then export RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/r01/librsmi.so; else unset RSMI_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o run --output-format csv -- python3 $R/bench.py $A > $O/prof_$lib.log 2>&1 || exit 3
done
echo ok
