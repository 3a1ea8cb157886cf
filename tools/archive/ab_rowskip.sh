# Syndrome reconstruct with the network restricted to the parity rows a
# pattern uses (this build) vs all rows (lib_ab/head); threshold re-check
# against the split-table kernel for small e.
set -o pipefail
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384 --pattern-pool 256"
HEAD=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/head/librsmi.so
for r in 1 2; do
  for e in 5 10 16; do
    echo "e=$e rowskip"; run $W --emin $e --emax $e --mode reconstruct || exit 1
    echo "e=$e all rows"; RSMI_LIB=$HEAD run $W --emin $e --emax $e --mode reconstruct || exit 1
  done
  for e in 2 3 4; do
    echo "e=$e rowskip syndrome"; RSMI_BITSLICE_REC_MIN_E=1 run $W --emin $e --emax $e --mode reconstruct || exit 1
    echo "e=$e split"; run $W --emin $e --emax $e --mode reconstruct || exit 1
  done
  echo "cfg5 rowskip"; run $W --emax 16 || exit 1
  echo "cfg5 head"; RSMI_LIB=$HEAD run $W --emax 16 || exit 1
done
