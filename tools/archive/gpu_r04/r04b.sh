#!/bin/bash
# GPU suite on the round-4 build (new: bench.py as child processes -- the
# N = 2 gloo rehearsal with the gather leg, the N = 1 config1/config5 legs;
# the pattern-wait watermark), then the config-5 reconstruct against its
# movement twin (gen_bitslice -x: same loads, stores, descriptors, no
# network / solve; lib_ab/mv) and one SQ pass of the shipped kernel.
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py $C5 "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['reconstruct_ms'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  for lib in cur mv; do
    one fresh $lib || exit 2
    one e16 $lib --emin 16 --emax 16 || exit 3
    one e4 $lib --emax 4 || exit 4
  done
done
cat $O/ab.log
unset RSMI_LIB
# config-1 latency: direct-staging host pipeline (default) vs the copy-engine path
L="--stripes 64 --shard 65536 --steps 2 --warmup 1 --cpu-seconds 0 --config1-reps 200 --config5-stripes 64 --config5-steps 1 --config5-warmup 1"
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py $L > $O/c1_direct_$rep.json 2>> $O/c1.err || exit 6
  RSMI_HOSTPIPE=dma timeout -k 10 200 python3 bench.py $L > $O/c1_dma_$rep.json 2>> $O/c1.err || exit 7
done
B="python3 bench.py --steps 2 --warmup 1 $C5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAVES --kernel-trace -d $O/pmc_sq/sq -o run --output-format csv -- $B > $O/sq.log 2>&1 || exit 5
echo done
