#!/bin/bash
# r06u: where a single message's mailbox jobs spend their time -- device
# wall-clock stamps per job (RSMI_MAILBOX_STAMPS) beside the host's post and
# done times and the phase trace; caller on the GPU's NUMA node.
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
for W in decode encode; do
  RSMI_PIN_GPU_NUMA=1 RSMI_MAILBOX_STAMPS=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_stamps.trace 2>&1 || { tail $O/${W}_stamps.trace; exit 2; }
  cat $O/${W}_stamps.trace
done
