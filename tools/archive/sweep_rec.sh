set -o pipefail
run() { timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -2 || exit 1
echo "both default"; run || exit 1
echo "rec parity 10-13"; run --mode reconstruct --erase 10,11,12,13 || exit 1
echo "rec data 0-3"; run --mode reconstruct --erase 0,1,2,3 || exit 1
echo "rec e=1"; run --mode reconstruct --emin 1 --emax 1 || exit 1
echo "rec e=4"; run --mode reconstruct --emin 4 --emax 4 || exit 1
echo "rec e=1..4"; run --mode reconstruct || exit 1
