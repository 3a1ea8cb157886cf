# Bit-sliced syndrome reconstruct (bitslice.hpp): GPU parity, then same-box
# A/B for RS(64,16) at BASELINE config 5 shapes: default (split by erasure
# count), all stripes through the syndrome kernel (RSMI_BITSLICE_REC_MIN_E=1)
# and all through the split-table kernel (RSMI_BITSLICE_REC=0).
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['reconstruct_ms'], b['reconstruct_kernel'])"; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --mode reconstruct"
for r in 1 2; do
  echo "RS(64,16) e=1..16 pool256 split";     run $W --pattern-pool 256 || exit 1
  echo "RS(64,16) e=1..16 pool256 bitslice";  RSMI_BITSLICE_REC_MIN_E=1 run $W --pattern-pool 256 || exit 1
  echo "RS(64,16) e=1..16 pool256 table";     RSMI_BITSLICE_REC=0 run $W --pattern-pool 256 || exit 1
done
echo "RS(64,16) e=1..16 fresh split";    run $W || exit 1
echo "RS(64,16) e=1..16 fresh table";    RSMI_BITSLICE_REC=0 run $W || exit 1
for e in 4 5 6; do
  echo "RS(64,16) e=$e bitslice"; RSMI_BITSLICE_REC_MIN_E=1 run $W --emin $e --emax $e --pattern-pool 256 || exit 1
  echo "RS(64,16) e=$e table";    RSMI_BITSLICE_REC=0 run $W --emin $e --emax $e --pattern-pool 256 || exit 1
done
echo "RS(64,16) both, default"; run --k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256 || exit 1
