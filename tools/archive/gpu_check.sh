set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -3 || exit 1
echo "RS(10,4) default"; run || exit 1
echo "RS(64,16) fully random patterns"; run --k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 || exit 1
echo "RS(64,16) pool 256"; run --k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 --pattern-pool 256 || exit 1
