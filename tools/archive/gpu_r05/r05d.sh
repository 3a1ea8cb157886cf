#!/bin/bash
# GPU suite with small bit-sliced calls routed to the split-table kernel;
# latency per stripe batch; config1 leg A/B of the bounded wait_event polling
# (default) vs polling every wait (RSMI_SYNC_ADAPTIVE=0); config-5 encode
# prefetch depth A/B (ep6/ep8), three interleaved reps.
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--batches 1,2,4,8,16,17,64,256"
timeout -k 10 200 python3 tools/bench_latency_sweep.py $B > $O/lat_rs64.json 2>> $O/lat.err || exit 2
timeout -k 10 200 python3 tools/bench_latency_sweep.py --k 10 --n 14 --shard 1048576 --batches 1,2,4,8,16,17,64 > $O/lat_rs10.json 2>> $O/lat.err || exit 3
L="--stripes 64 --shard 65536 --steps 2 --warmup 1 --cpu-seconds 0 --config1-reps 60 --config5-stripes 64 --config5-steps 1 --config5-warmup 1"
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py $L > $O/c1_adaptive_$rep.json 2>> $O/c1.err || exit 4
  RSMI_SYNC_ADAPTIVE=0 timeout -k 10 200 python3 bench.py $L > $O/c1_poll_$rep.json 2>> $O/c1.err || exit 5
done
for f in $O/c1_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); c=d['config1']; print('$f', c['codec'].get('encode_ms'), c['codec'].get('decode4_ms'), c['codec'].get('decode4_arena_ms'), c['codec'].get('decode4_batch64_ms_per_message'), c['plugin'])"; done
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode both --cpu-seconds 0 --no-extra-legs --steps 8 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['encode_GBps'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2 3; do
  for lib in cur ep6 ep8; do
    one fresh $lib $C5 || exit 6
  done
done
unset RSMI_LIB
cat $O/ab.log
echo done
