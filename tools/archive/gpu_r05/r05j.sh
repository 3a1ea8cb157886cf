#!/bin/bash
# stream_probe: one config-1-sized pageable message through staging + one
# kernel, in the engine's two-launch shape vs one launch fed by per-group
# ready flags (host copy overlapping the kernel's PCIe reads).
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 120 ./tools/stream_probe > $O/stream_probe.log 2>&1 || { cat $O/stream_probe.log; exit 1; }
cat $O/stream_probe.log
