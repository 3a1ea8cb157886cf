# Bit-sliced RS(64,16) encode vs its movement-only twins: -x (same registers,
# 2 waves/SIMD) and -X (57 VGPRs, 8 waves/SIMD): does occupancy bound the
# kernel's memory rate?
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 --mode encode "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(b['encode_GBps'], b['encode_ms'], b['encode_kernel'])"; }
L=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab
W="--k 64 --n 80 --shard 65536 --stripes 16384"
for r in 1 2; do
  echo "bitslice";        run $W || exit 1
  echo "movement -x";     RSMI_LIB=$L/move/librsmi.so run $W || exit 1
  echo "movement -X";     RSMI_LIB=$L/movelow/librsmi.so run $W || exit 1
  echo "split-table K64_MG16"; RSMI_BITSLICE=0 run $W || exit 1
done
