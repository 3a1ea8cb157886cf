# r02av: SQ counters of the config-5 kernels with the XCD-aware order
# (16 erasures and the 1-16 mix, fresh patterns) and of the RS(10,4) headline.
set -o pipefail
R=$GRAFT_REPO_ROOT
PMC_TAG=r02av_cfg5_e16 BENCH_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emin 16 --emax 16" bash $R/tools/pmc_valu.sh || exit 1
PMC_TAG=r02av_cfg5_mix BENCH_ARGS="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16" bash $R/tools/pmc_valu.sh || exit 2
PMC_TAG=r02av_headline BENCH_ARGS="" bash $R/tools/pmc_valu.sh || exit 3
echo ok
