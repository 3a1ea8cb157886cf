# A/B of the syndrome-kernel solve (8-row output groups with fields computed
# once per group, row-at-a-time tables) against the previous build
# (lib_ab/${AB_BASE:-r02pre}), config-5 shapes, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${AB_TAG:-r02l}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py -k "bitslice or wide_code or reconstruct_ptrs or split_between" -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
run() { timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['reconstruct_ms'])"; }
C="--k 64 --n 80 --shard 65536 --stripes 16384"
for rep in 1 2; do
  for lib in cur base; do
    if [ $lib = base ]; then export RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/${AB_BASE:-r02pre}/librsmi.so; else unset RSMI_LIB; fi
    echo "== $lib rep $rep: e=16 fresh" >> $O/ab.log; run $C --emin 16 --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== $lib rep $rep: e=1..16 fresh" >> $O/ab.log; run $C --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 3
    echo "== $lib rep $rep: e=1..16 pool 256" >> $O/ab.log; run $C --emax 16 --pattern-pool 256 >> $O/ab.log 2>> $O/ab.err || exit 4
    echo "== $lib rep $rep: e=5..8 fresh" >> $O/ab.log; run $C --emin 5 --emax 8 >> $O/ab.log 2>> $O/ab.err || exit 5
  done
done
echo ok
