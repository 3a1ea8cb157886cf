# Syndrome reconstruct prefetch depth (gen_bitslice -P): default build
# (4, as the encode) vs lib_ab/P6 and lib_ab/P8, RS(64,16) config 5 shapes.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
W="--k 64 --n 80 --shard 65536 --stripes 16384"
L=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab
for r in 1 2; do
  for v in base P6 P8; do
    if [ $v = base ]; then export RSMI_LIB=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib/librsmi.so; else export RSMI_LIB=$L/$v/librsmi.so; fi
    echo "$v e=4"; run $W --emin 4 --emax 4 --pattern-pool 256 --mode reconstruct || exit 1
    echo "$v e=16"; run $W --emin 16 --emax 16 --pattern-pool 256 --mode reconstruct || exit 1
    echo "$v cfg5 pool"; run $W --emax 16 --pattern-pool 256 --mode reconstruct || exit 1
  done
done
