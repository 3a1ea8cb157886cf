# GPU parity, then the syndrome reconstruct kernel with unconditional
# (prefetched) loads vs the build before (lib_ab/mg16: loads under a branch).
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384"
OLD=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/mg16/librsmi.so
for r in 1 2; do
  for e in 5 10 16; do
    echo "e=$e new"; run $W --emin $e --emax $e --pattern-pool 256 --mode reconstruct || exit 1
    echo "e=$e old"; RSMI_LIB=$OLD run $W --emin $e --emax $e --pattern-pool 256 --mode reconstruct || exit 1
  done
  echo "cfg5 pool new"; run $W --emax 16 --pattern-pool 256 || exit 1
  echo "cfg5 fresh new"; run $W --emax 16 || exit 1
done
