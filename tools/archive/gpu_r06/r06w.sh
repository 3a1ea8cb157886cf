#!/bin/bash
# r06w: chunk splits with the jobs' arguments in the kernel arguments; the
# GPU now finishes ~15 us after the last post, so a smaller last chunk may
# pay.  Caller on the GPU's NUMA node, interleaved processes.
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_${name}_$rep.trace 2>&1 || { tail $O/${W}_${name}_$rep.trace; exit 2; }
}
for rep in 1 2 3; do
  for W in decode encode; do
    run s25_60 RSMI_CHUNK_SPLIT=25,60
    run s30_65 RSMI_CHUNK_SPLIT=30,65
    run s20_50_80 RSMI_CHUNK_SPLIT=20,50,80
    run s25_55_80 RSMI_CHUNK_SPLIT=25,55,80
    run s20_45_75 RSMI_CHUNK_SPLIT=20,45,75
  done
done
for f in $O/*.trace; do echo "$f: $(grep -h 'median' $f | grep -v RSMI | sed 's/ over 1000 calls.*//')"; done
