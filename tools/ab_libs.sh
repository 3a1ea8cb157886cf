#!/bin/bash
# Same-box A/B of engine builds (lib_ab/<name>/librsmi.so; "cur" = lib/),
# config-5 reconstruct shapes, interleaved.  AB_TAG names the output dir,
# AB_LIBS the builds, AB_MODE the bench mode, AB_REPS the repetitions.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${AB_TAG:-ab}
mkdir -p $O
run() { timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --mode ${AB_MODE:-reconstruct} "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_ms'], b['reconstruct_ms'])"; }
C="--k 64 --n 80 --shard 65536 --stripes 16384"
for rep in $(seq ${AB_REPS:-2}); do
  for lib in ${AB_LIBS:-cur}; do
    if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
    echo "== $lib rep $rep: e=16 fresh" >> $O/ab.log; run $C --emin 16 --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== $lib rep $rep: e=1..16 fresh" >> $O/ab.log; run $C --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 3
    echo "== $lib rep $rep: e=1..16 pool 256" >> $O/ab.log; run $C --emax 16 --pattern-pool 256 >> $O/ab.log 2>> $O/ab.err || exit 4
    echo "== $lib rep $rep: e=1..4 fresh" >> $O/ab.log; run $C --emax 4 >> $O/ab.log 2>> $O/ab.err || exit 5
  done
done
echo ok
