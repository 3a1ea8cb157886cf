# Bit-sliced encode vs its movement-only twin (lib_ab/move: same loads,
# stores and block shape, no transpose or network): how far the coding work
# keeps the kernel from its own access pattern's memory rate.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 --mode encode "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(b['encode_GBps'], b['encode_ms'], b['encode_kernel'])"; }
MOVE=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/move/librsmi.so
W="--k 64 --n 80 --shard 65536 --stripes 16384"
for r in 1 2; do
  echo "RS(64,16) bitslice"; run $W || exit 1
  echo "RS(64,16) movement"; RSMI_LIB=$MOVE run $W || exit 1
  echo "RS(10,4) bitslice"; RSMI_BITSLICE=1 run || exit 1
  echo "RS(10,4) movement"; RSMI_BITSLICE=1 RSMI_LIB=$MOVE run || exit 1
  echo "RS(10,4) split-table"; run || exit 1
done
# K64 split-table kernels: double-buffered survivor batches (this build) vs
# single-buffered (lib_ab/prev), 1-4 erasures (all stripes on K64_MG4).
PREV=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/prev/librsmi.so
rrun() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --mode reconstruct "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(b['reconstruct_GBps'], b['reconstruct_ms'])"; }
for r in 1 2; do
  echo "K64_MG4 e=1..4 double-buffered"; rrun $W --emax 4 --pattern-pool 256 || exit 1
  echo "K64_MG4 e=1..4 single";          RSMI_LIB=$PREV rrun $W --emax 4 --pattern-pool 256 || exit 1
  echo "RS(10,4) headline rec";          rrun || exit 1
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
