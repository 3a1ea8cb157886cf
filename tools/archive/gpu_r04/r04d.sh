#!/bin/bash
# Config-5 syndrome reconstruct: the shipped kernel (buffer loads since
# r04c) against BL = -B -L (no padded outputs in the last solve group);
# then the config-1 latency breakdown (tools/probe_latency.py) with and
# without the copy-pool spin.
# First the bit-sliced parity tests under each variant (RSMI_LIB), then a
# same-box A/B, reconstruct only, 10 steps, 2 interleaved reps.
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
for lib in BL; do
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
  for lib in cur BL; do
    one fresh $lib $C5 || exit 2
    one e16 $lib $C5 --emin 16 --emax 16 || exit 3
    one e8 $lib $C5 --emin 5 --emax 8 || exit 4
    one pool $lib $C5 --pattern-pool 256 || exit 5
    one rs8_14 $lib --k 8 --n 14 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2 || exit 6
  done
done
unset RSMI_LIB
cat $O/ab.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || exit 7
  RSMI_COPY_SPIN_US=100 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_spin_$rep.json 2>> $O/probe.err || exit 8
done
cat $O/probe_*.json
echo done
