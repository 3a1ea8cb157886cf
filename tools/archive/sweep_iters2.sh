# Strided block iterations (iteration it codes chunk it*chunks+chunk): parity
# under RSMI_ITERS=3, then the headline bench at 1/2/4 iterations.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'])"; }
RSMI_ITERS=3 timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -2 || exit 1
for r in 1 2; do
  for it in 1 2 4; do echo "iters=$it"; RSMI_ITERS=$it run || exit 1; done
done
