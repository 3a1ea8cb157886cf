# Same-box A/B of the bit-sliced kernels' load prefetch depth: builds in
# noise-erasurecode-plugin_amd/lib_ab/pf<N> (make BITSLICE_PREFETCH=N, on the CPU
# beforehand, N = 2 3 4 6), selected with RSMI_LIB.  RS(64,16) encode and reconstruct.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
W="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256"
for r in 1 2; do
  for pf in 2 3 4 6; do
    echo "prefetch $pf"; RSMI_LIB=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/pf$pf/librsmi.so run $W || exit 1
  done
done
