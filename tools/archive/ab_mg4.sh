# GPU parity, then RS(64,16) reconstruct with 1-4 erasures per stripe (all on
# the split-table kernel) and config 5: K64_MG4 (this build) vs K64_MG16
# (lib_ab/mg16, the build before the MG4 variant).
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384"
for r in 1 2; do
  echo "e 1-4 MG4";  run $W --emax 4 --pattern-pool 256 || exit 1
  echo "e 1-4 MG16"; RSMI_LIB=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/mg16/librsmi.so run $W --emax 4 --pattern-pool 256 || exit 1
  echo "cfg5 pool MG4";  run $W --emax 16 --pattern-pool 256 || exit 1
  echo "cfg5 pool MG16"; RSMI_LIB=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/mg16/librsmi.so run $W --emax 16 --pattern-pool 256 || exit 1
done
