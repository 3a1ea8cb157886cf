# GPU parity; syndrome reconstruct with absent inputs loading a zero page
# (this build) vs re-reading the previous input (lib_ab/prev); then FETCH_SIZE
# of both on config 5 (absent-input loads should cost no HBM reads).
set -o pipefail
export TMPDIR=/tmp
run() { timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'])"; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
W="--k 64 --n 80 --shard 65536 --stripes 16384"
PREV=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/prev/librsmi.so
for r in 1 2; do
  echo "e=10 zpage"; run $W --emin 10 --emax 10 --pattern-pool 256 --mode reconstruct || exit 1
  echo "e=10 prev";  RSMI_LIB=$PREV run $W --emin 10 --emax 10 --pattern-pool 256 --mode reconstruct || exit 1
  echo "cfg5 zpage"; run $W --emax 16 --pattern-pool 256 || exit 1
  echo "cfg5 prev";  RSMI_LIB=$PREV run $W --emax 16 --pattern-pool 256 || exit 1
done
O=$GRAFT_REPO_ROOT/gpurun_out/zpage_fetch
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/new -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 $W --emin 10 --emax 10 --pattern-pool 256 --mode reconstruct > $O/new.log 2>&1 || exit 2
echo fetch-done
