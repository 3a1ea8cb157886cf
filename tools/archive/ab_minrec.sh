# Threshold between the split-table and the (row-skipping) syndrome
# reconstruct: e=1 both ways, config 5 with RSMI_BITSLICE_REC_MIN_E 2/3/5.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
W="--k 64 --n 80 --shard 65536 --stripes 16384"
for r in 1 2; do
  echo "e=1 syndrome"; RSMI_BITSLICE_REC_MIN_E=1 run $W --pattern-pool 256 --emin 1 --emax 1 --mode reconstruct || exit 1
  echo "e=1 split"; RSMI_BITSLICE_REC_MIN_E=99 run $W --pattern-pool 256 --emin 1 --emax 1 --mode reconstruct || exit 1
  for me in 1 2 3 5; do
    echo "cfg5 pool min_e=$me"; RSMI_BITSLICE_REC_MIN_E=$me run $W --pattern-pool 256 --emax 16 || exit 1
  done
  echo "cfg5 fresh min_e=2"; RSMI_BITSLICE_REC_MIN_E=2 run $W --emax 16 || exit 1
  echo "cfg5 fresh min_e=5"; RSMI_BITSLICE_REC_MIN_E=5 run $W --emax 16 || exit 1
done
