# r02i: RS(8,14) with the 6-row group (K8_MG6) vs the round-1 build, its
# parity test, and the BLAKE2b bench after the binding / copy-pool changes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py -k "rs8_14 or encode_matches_oracle or stripes_matches_oracle" -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
run() { timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'], b['encode_kernel'], b['reconstruct_kernel'])"; }
for rep in 1 2; do
  for lib in cur r01; do
    if [ $lib = r01 ]; then export RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/r01/librsmi.so; else unset RSMI_LIB; fi
    echo "== $lib rep $rep: RS(8,14) S=1M 4096 stripes" >> $O/ab.log; run --k 8 --n 14 --stripes 4096 >> $O/ab.log 2>> $O/ab.err || exit 2
  done
done
unset RSMI_LIB
timeout -k 10 300 python3 $R/tools/bench_blake2b.py > $O/blake2b.json 2> $O/blake2b.err || exit 3
echo ok
