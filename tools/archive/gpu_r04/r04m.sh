#!/bin/bash
# Syndrome solve in row pairs (gen_bitslice -C, lib_ab/C) and pairs plus a
# padding-free last output group (-C -D, lib_ab/CD): the bit-sliced parity
# tests on both builds, then reconstruct-only A/B against the shipped solve,
# 10 steps x 2, config-5 shapes and RS(8,14).
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/noise-erasurecode-plugin_amd/lib_ab
for lib in C CD; do
  RSMI_LIB=$L/$lib/librsmi.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "bitslice or row_subset or config5 or xcd" > $O/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 $O/pytest_$lib.log; exit 1; }
  tail -1 $O/pytest_$lib.log
done
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$L/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  for lib in cur C CD; do
    one fresh $lib $C5 || exit 2
    one e16 $lib $C5 --emin 16 --emax 16 || exit 3
    one e8 $lib $C5 --emin 5 --emax 8 || exit 4
    one pool $lib $C5 --pattern-pool 256 || exit 5
    one rs8_14 $lib --k 8 --n 14 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2 || exit 6
  done
done
unset RSMI_LIB
cat $O/ab.log
echo done
