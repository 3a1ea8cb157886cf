#!/bin/bash
# GPU suite on the current build (split-table prologue: survivor ids and
# addresses in batches; bit-sliced buffer range 4 GiB + the past-2-GiB test);
# membench10 with prefetch depth and reads-only variants; real-kernel A/B of
# the config-5 bit-sliced prefetch depth (rp6/rp8: reconstruct 6/8; ep6/ep8:
# encode and reconstruct 6/8) and of the RS(10,4) prologue (base = round 4).
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./tools/membench10 16384 1 16 > $O/mb10_fresh.log 2>&1 || exit 2
timeout -k 10 120 ./tools/membench10 16384 1 4 > $O/mb10_e1_4.log 2>&1 || exit 3
cat $O/mb10_*.log
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode both --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['encode_GBps'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  for lib in cur rp6 rp8 ep6 ep8; do
    one fresh $lib $C5 || exit 4
    one e16 $lib $C5 --emin 16 --emax 16 || exit 5
    one e1_4 $lib $C5 --emax 4 || exit 6
  done
  for lib in base cur; do
    one headline $lib --mode both --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2 || exit 7
  done
done
unset RSMI_LIB
cat $O/ab.log
echo done
