# GPU parity, then config-5 reconstruct with a fresh pattern per stripe:
# structured d x d decode rows (default) vs whole-matrix Gauss-Jordan.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384 --emax 16"
for r in 1 2; do
  echo "RS(64,16) fresh patterns, structured"; run $W || exit 1
  echo "RS(64,16) fresh patterns, generic";    RSMI_INVERT_GENERIC=1 run $W || exit 1
done
echo "RS(10,4) default"; run || exit 1
