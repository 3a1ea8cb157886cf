# Generated bit-sliced encode kernel: GPU parity, then same-box A/B against
# the split-table kernel (RSMI_BITSLICE=0/1) for RS(64,16) and RS(10,4).
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['encode_kernel'])"; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -3 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256"
for r in 1 2; do
  echo "RS(64,16) bitslice"; run $W --mode encode || exit 1
  echo "RS(64,16) table";    RSMI_BITSLICE=0 run $W --mode encode || exit 1
done
echo "RS(10,4) bitslice"; RSMI_BITSLICE=1 run --mode encode || exit 1
echo "RS(10,4) table";    run --mode encode || exit 1
