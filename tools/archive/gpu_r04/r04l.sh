#!/bin/bash
# Column-chunked staging of small host-API messages (the second half staged
# while the kernel codes the first): GPU suite, then the latency probe with
# 1 / 2 (default for >= 256 KiB) / 3 chunks; then the row-guard granularity
# A/B of the syndrome kernel (G1 / G4 = one guard per row / per 4 rows,
# gen_bitslice -G; shipped: groups of 2), reconstruct only, 10 steps x 2.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for nch in 1 2 3; do
    RSMI_STAGE_CHUNKS=$nch timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_c${nch}_$rep.json 2>> $O/probe.err || exit 2
  done
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['reconstruct_GBps'])" >> $O/ab.log
}
for lib in G1 G4; do
  RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "bitslice or row_subset or config5 or xcd" > $O/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 $O/pytest_$lib.log; exit 1; }
  tail -1 $O/pytest_$lib.log
done
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1 lib=$2; shift 2
  if [ $lib = cur ]; then unset RSMI_LIB; else export RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/$lib/librsmi.so; fi
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag $lib', b['encode_ms'], b['reconstruct_ms'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  for lib in cur G1 G4; do
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
