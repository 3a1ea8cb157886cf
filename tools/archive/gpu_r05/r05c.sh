#!/bin/bash
# GPU suite on the current build (batched split-table prologue, dynamic row
# count, inline descriptors for small calls, 4 GiB buffer range + the
# past-2-GiB test, decode overlap, watermark and -M diagnostic tests, the C++
# plugin harness); membench10 prefetch/reads variants; config-5 bit-sliced
# prefetch depth A/B (rp6/rp8: reconstruct 6/8; ep6/ep8: both 6/8); RS(10,4)
# headline A/B (base = round 4, nodyn = this build without the dynamic row
# count); latency per stripe batch; the default line.
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./tools/membench10 16384 1 16 > $O/mb10_fresh.log 2>&1 || exit 2
timeout -k 10 120 ./tools/membench10 16384 1 4 > $O/mb10_e1_4.log 2>&1 || exit 3
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode both --cpu-seconds 0 --no-extra-legs --steps 8 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['encode_GBps'], b['reconstruct_GBps'])" >> $O/ab.log
}
for lib in cur rp6 rp8 ep6 ep8; do
  one fresh $lib $C5 || exit 4
  one e16 $lib $C5 --emin 16 --emax 16 || exit 5
  one e1_4 $lib $C5 --emax 4 || exit 6
done
for rep in 1 2; do
  for lib in base nodyn cur; do
    one headline $lib --mode both --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2 || exit 7
  done
done
unset RSMI_LIB
cat $O/ab.log
B="--batches 1,2,4,8,16,17,64,256"
timeout -k 10 200 python3 tools/bench_latency_sweep.py $B > $O/lat_default.json 2>> $O/lat.err || exit 8
RSMI_NO_INLINE_DESC=1 timeout -k 10 200 python3 tools/bench_latency_sweep.py $B > $O/lat_upload.json 2>> $O/lat.err || exit 9
RSMI_BITSLICE_REC=0 timeout -k 10 200 python3 tools/bench_latency_sweep.py $B > $O/lat_recsplit.json 2>> $O/lat.err || exit 10
RSMI_BITSLICE=0 RSMI_BITSLICE_REC=0 timeout -k 10 200 python3 tools/bench_latency_sweep.py $B > $O/lat_split.json 2>> $O/lat.err || exit 11
timeout -k 10 200 python3 tools/bench_latency_sweep.py --k 10 --n 14 --shard 1048576 --batches 1,2,4,8,16,17,64 > $O/lat_rs10.json 2>> $O/lat.err || exit 12
RSMI_NO_INLINE_DESC=1 timeout -k 10 200 python3 tools/bench_latency_sweep.py --k 10 --n 14 --shard 1048576 --batches 1,2,4,8,16,17,64 > $O/lat_rs10_upload.json 2>> $O/lat.err || exit 13
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 14; }
cat $O/bench.json
echo done
