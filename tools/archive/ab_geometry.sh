# Column geometry of the bit-sliced kernels: 0 (wave owns a 2 KiB window,
# this build) vs 1 (each block-wide load instruction covers 4 KiB,
# lib_ab/geo1), real kernels and movement-only twins (lib_ab/move, movegeo1).
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
L=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab
W="--k 64 --n 80 --shard 65536 --stripes 16384"
RSMI_LIB=$L/geo1/librsmi.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bitslice or wide" --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for r in 1 2; do
  echo "cfg5 geo0"; run $W --emax 16 --pattern-pool 256 || exit 1
  echo "cfg5 geo1"; RSMI_LIB=$L/geo1/librsmi.so run $W --emax 16 --pattern-pool 256 || exit 1
  echo "enc move geo0"; RSMI_LIB=$L/move/librsmi.so run $W --mode encode || exit 1
  echo "enc move geo1"; RSMI_LIB=$L/movegeo1/librsmi.so run $W --mode encode || exit 1
  echo "RS(10,4) bitslice geo0"; RSMI_BITSLICE=1 run --mode encode || exit 1
  echo "RS(10,4) bitslice geo1"; RSMI_BITSLICE=1 RSMI_LIB=$L/geo1/librsmi.so run --mode encode || exit 1
done
