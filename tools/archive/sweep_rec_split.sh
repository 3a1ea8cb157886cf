# RS(64,16), 64 KiB shards: fixed e erasures per stripe, split-table kernel
# (K64_MG4/MG8/MG16 by e) vs the bit-sliced syndrome kernel, to place
# RSMI_BITSLICE_REC_MIN_E.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --mode reconstruct "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(b['reconstruct_GBps'], b['reconstruct_ms'])"; }
W="--k 64 --n 80 --shard 65536 --stripes 16384 --pattern-pool 256"
for e in 4 5 6 7 8 9 10 12; do
  echo "e=$e split";    RSMI_BITSLICE_REC_MIN_E=99 run $W --emin $e --emax $e || exit 1
  echo "e=$e syndrome"; RSMI_BITSLICE_REC_MIN_E=1 run $W --emin $e --emax $e || exit 1
done
