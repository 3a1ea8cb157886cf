#!/bin/bash
# r06ar: where the arena (in-place) decode's time goes: phases, and with the
# grid (three chunks) its device stamps.
set -o pipefail
O=gpurun_out/r06ar
mkdir -p $O
export TMPDIR=/tmp
RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py decode_arena 1000 > $O/arena.trace 2>&1 || { tail $O/arena.trace; exit 1; }
RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 RSMI_INPLACE_CHUNKS=1 timeout -k 10 120 python3 tools/trace_single.py decode_arena 1000 > $O/arena_chunks.trace 2>&1 || { tail $O/arena_chunks.trace; exit 1; }
RSMI_PIN_GPU_NUMA=1 RSMI_MAILBOX_STAMPS=1 RSMI_INPLACE_CHUNKS=1 timeout -k 10 120 python3 tools/trace_single.py decode_arena 1000 > $O/arena_stamps.trace 2>&1 || { tail $O/arena_stamps.trace; exit 1; }
RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py decode 1000 > $O/decode.trace 2>&1 || { tail $O/decode.trace; exit 1; }
cat $O/arena.trace $O/arena_chunks.trace $O/arena_stamps.trace $O/decode.trace | grep -v amdgpu.ids
