# r01e measurements: the default bench line (headline, CPU baseline included),
# then the other BASELINE configs and worst cases with short runs.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'], d['roofline']['frac'])"; }
echo "default bench.py line"; timeout -k 10 400 python3 bench.py || exit 1
echo "RS(10,4) 4 data erasures every stripe"; run --erase 0,1,2,3 || exit 1
echo "RS(10,4) 4 parity erasures every stripe"; run --erase 10,11,12,13 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384"
echo "RS(64,16) e=1..16 pool 256"; run $W --emax 16 --pattern-pool 256 || exit 1
echo "RS(64,16) e=1..16 fresh"; run $W --emax 16 || exit 1
echo "RS(64,16) e=16 fresh"; run $W --emin 16 --emax 16 || exit 1
echo "RS(64,16) e=1..4 fresh"; run $W --emax 4 || exit 1
echo "RS(4,2) S=1M 8192 stripes"; run --k 4 --n 6 --stripes 8192 || exit 1
echo "RS(8,14) S=1M 4096 stripes"; run --k 8 --n 14 --stripes 4096 || exit 1
