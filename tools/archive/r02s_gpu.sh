#!/bin/bash
# r02s: syndrome kernel without the parity-survivor transpose (A/B vs the
# r02r build) on config-5 shapes; parity tests of the bit-sliced paths.
set -euo pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bitslice or rec or config5 or cfg5 or reconstruct" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
B="python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 6 --warmup 2"
for rep in 1 2; do
for lib in noise-erasurecode-plugin_amd/lib_ab/r02r/librsmi.so noise-erasurecode-plugin_amd/lib/librsmi.so; do
  tag=$(basename $(dirname $lib))
  RSMI_LIB=$R/$lib timeout -k 10 240 $B --pattern-pool 256 > $O/mix_pool_${tag}_$rep.json 2>> $O/err.log
  RSMI_LIB=$R/$lib timeout -k 10 240 $B --emin 16 --emax 16 > $O/e16_${tag}_$rep.json 2>> $O/err.log
  RSMI_LIB=$R/$lib timeout -k 10 240 $B > $O/mix_fresh_${tag}_$rep.json 2>> $O/err.log
done
done
echo ab done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fresh -o run --output-format csv -- python3 bench.py --k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --steps 6 --warmup 2 > $O/prof_fresh.log 2>&1
echo prof done
