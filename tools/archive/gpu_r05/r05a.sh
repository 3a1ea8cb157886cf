#!/bin/bash
# Config-5 syndrome reconstruct: the round-4 build (lib_ab/base) against the
# prologue fix (solve coefficients built into LDS after the last input, no
# vmcnt(0) drain of the first inputs' loads); the movement twins of both
# (gen_bitslice -x: lib_ab/mvold, lib_ab/mvnew).  GPU suite on the new build first.
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  for lib in base cur mvold mvnew; do
    one fresh $lib $C5 || exit 2
    one e16 $lib $C5 --emin 16 --emax 16 || exit 3
    one e1_4 $lib $C5 --emax 4 || exit 4
  done
  for lib in base cur; do
    one rs8_14 $lib --k 8 --n 14 --mode both --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2 || exit 5
  done
done
unset RSMI_LIB
# Headline RS(10,4) reconstruct: pattern-sorted descriptors (patterns are
# numbered by erasure count, so the launch runs e = 1, 2, 3, 4 phases) vs
# address order (RSMI_NO_SORT).
H="--mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
for rep in 1 2; do
  one h_sorted cur $H || exit 6
  RSMI_NO_SORT=1 one h_nosort cur $H || exit 7
done
cat $O/ab.log
echo done
