# Same-box A/B of the non-temporal cache policy (RSMI_NT) on the headline
# workload, after the GPU parity suite.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'])"; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -3 || exit 1
for r in 1 2; do
  echo "nt";       run || exit 1
  echo "temporal"; RSMI_NT=0 run || exit 1
done
echo "RS(4,2) nt"; run --k 4 --n 6 --stripes 8192 --mode encode || exit 1
echo "RS(64,16) nt"; run --k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256 || exit 1
