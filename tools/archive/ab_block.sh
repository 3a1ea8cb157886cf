set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'])"; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q 2>&1 | tail -1 || exit 1
for r in 1 2; do
  for bt in 256 512 1024; do echo "block=$bt"; RSMI_BLOCK=$bt run || exit 1; done
done
echo "e=1 256"; RSMI_BLOCK=256 run --mode reconstruct --emin 1 --emax 1 || exit 1
echo "e=1 512"; RSMI_BLOCK=512 run --mode reconstruct --emin 1 --emax 1 || exit 1
timeout -k 10 600 python3 tools/bench_host_api.py > gpurun_out/host_api3.log 2>&1 || exit 1
