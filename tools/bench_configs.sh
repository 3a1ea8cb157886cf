set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'], d['roofline']['frac'])"; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -2 || exit 1
echo "RS(64,16) S=64K 16384 stripes, e=1..16"; run --k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 || exit 1
echo "RS(64,16) e=16"; run --k 64 --n 80 --shard 65536 --stripes 16384 --emin 16 --emax 16 || exit 1
echo "RS(4,2) S=1M 8192 stripes"; run --k 4 --n 6 --stripes 8192 || exit 1
echo "RS(8,14) S=1M 4096 stripes"; run --k 8 --n 14 --stripes 4096 || exit 1
echo "RS(10,4) default"; run || exit 1
