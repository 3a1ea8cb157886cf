#!/bin/bash
# Config-5 syndrome reconstruct: shipped build vs gen_bitslice -B (buffer
# loads; absent inputs read an empty buffer range instead of the zero page);
# config-1 host-API latency variants of the direct host pipeline (chunking,
# copy-pool spin); the GPU suite on the new host-path build.
set -o pipefail
O=gpurun_out/r04c
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
  for lib in cur B; do
    one fresh $lib $C5 || exit 2
    one e16 $lib $C5 --emin 16 --emax 16 || exit 3
    one rs8_14 $lib --k 8 --n 14 --mode both --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2 || exit 4
  done
done
unset RSMI_LIB
cat $O/ab.log
L="--stripes 64 --shard 65536 --steps 2 --warmup 1 --cpu-seconds 0 --config1-reps 300 --config5-stripes 64 --config5-steps 1 --config5-warmup 1"
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py $L > $O/c1_base_$rep.json 2>> $O/c1.err || exit 6
  RSMI_COPY_SPIN_US=100 timeout -k 10 200 python3 bench.py $L > $O/c1_spin_$rep.json 2>> $O/c1.err || exit 7
  RSMI_HOSTPIPE_CHUNK=262144 timeout -k 10 200 python3 bench.py $L > $O/c1_chunk_$rep.json 2>> $O/c1.err || exit 8
  RSMI_HOSTPIPE_CHUNK=262144 RSMI_COPY_SPIN_US=100 timeout -k 10 200 python3 bench.py $L > $O/c1_chunkspin_$rep.json 2>> $O/c1.err || exit 9
done
for f in $O/c1_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); c=d['config1']; print('$f', c.get('codec'), c.get('cpu_1t',{}).get('avx2_1t'))"; done
echo done
