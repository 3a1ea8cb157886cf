# r02b: concurrency A/B on one context (round-1 library vs leases, and
# leases capped at 1) + SQ counters of the config-5 syndrome reconstruct.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 120 python3 $R/tools/bench_concurrency.py > $O/r02b_conc_leases.json 2> $O/r02b_conc.err || exit 1
RSMI_MAX_LEASES=1 timeout -k 10 120 python3 $R/tools/bench_concurrency.py > $O/r02b_conc_lease1.json 2>> $O/r02b_conc.err || exit 2
RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/r01/librsmi.so timeout -k 10 120 python3 $R/tools/bench_concurrency.py > $O/r02b_conc_r01.json 2>> $O/r02b_conc.err || exit 3
PMC_TAG=r02b_cfg5_e16 BENCH_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emin 16 --emax 16" bash $R/tools/pmc_valu.sh || exit 4
PMC_TAG=r02b_cfg5_mix BENCH_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16" bash $R/tools/pmc_valu.sh || exit 5
echo ok
