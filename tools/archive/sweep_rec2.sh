# Reconstruct shapes vs encode with the nt kernel (same box): isolates the
# descriptor path (parity 10-13 = encode's shape), e=1 data/parity, mixed.
set -o pipefail
run() { timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
echo "encode";           run --mode encode || exit 1
echo "rec parity 10-13"; run --mode reconstruct --erase 10,11,12,13 || exit 1
echo "rec data 0-3";     run --mode reconstruct --erase 0,1,2,3 || exit 1
echo "rec e=1 (13)";     run --mode reconstruct --erase 13 || exit 1
echo "rec e=1 (0)";      run --mode reconstruct --erase 0 || exit 1
echo "rec e=1 random";   run --mode reconstruct --emin 1 --emax 1 || exit 1
echo "rec e=4 random";   run --mode reconstruct --emin 4 --emax 4 || exit 1
echo "rec e=1..4";       run --mode reconstruct || exit 1
echo "both";             run || exit 1
