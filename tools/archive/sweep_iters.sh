set -o pipefail
for it in 1 2 4 8 16 64; do
  echo "iters=$it"
  RSMI_ITERS=$it timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['breakdown']['encode_GBps'], d['breakdown']['reconstruct_GBps'])" || exit 1
done
