set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'])"; }
for r in 1 2; do
  echo "sorted";   run --mode reconstruct || exit 1
  echo "unsorted"; RSMI_NO_SORT=1 run --mode reconstruct || exit 1
done
