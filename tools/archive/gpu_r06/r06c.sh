#!/bin/bash
# r06c: config-5 A/B of generator options on the syndrome reconstruct and the
# bit-sliced encode: 64-bit transpose shifts (-W), the solve tail (-L: no
# padded outputs in the last group), both; plus the SQ pass of the shipped
# kernel on three mixes (VALU per wave for tools/valu_model.py).
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
AB_TAG=r06c AB_LIBS="cur shift64 tail tailW" AB_REPS=2 timeout -k 10 900 bash tools/ab_libs.sh || { echo "ab failed"; tail $O/ab.err; exit 2; }
# encode too (bit-sliced encode uses the same transpose)
for lib in cur shift64; do
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  for rep in 1 2; do
    echo "== $lib encode rep $rep" >> $O/enc.log
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extra-legs --mode encode --k 64 --n 80 --shard 65536 --stripes 16384 2>>$O/enc.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['breakdown']['encode_ms'])" >> $O/enc.log || exit 3
  done
done
unset RSMI_LIB
for mix in "fresh:--emax 16" "e16:--emin 16 --emax 16" "e4:--emax 4"; do
  tag=${mix%%:*}; args=${mix#*:}
  PMC_TAG=r06c_$tag BENCH_ARGS="--no-extra-legs --mode reconstruct --k 64 --n 80 --shard 65536 --stripes 16384 $args" timeout -k 10 300 bash tools/pmc_valu.sh > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; exit 4; }
done
python3 tools/sq_summary.py gpurun_out/pmc_r06c_fresh gpurun_out/pmc_r06c_e16 gpurun_out/pmc_r06c_e4 > $O/sq_summary.md 2>&1
cat $O/ab.log $O/enc.log $O/sq_summary.md
