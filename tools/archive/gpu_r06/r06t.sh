#!/bin/bash
# r06t: how the present data shares reach dst during a single decode --
# the copy pool's async job (default) vs the caller alone (memcpy) vs the
# caller alone with streaming stores; caller on the GPU's NUMA node.
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_${name}_$rep.trace 2>&1 || { tail $O/${W}_${name}_$rep.trace; exit 2; }
}
W=decode
for rep in 1 2 3; do
  run pool RSMI_PRESENT_COPY=pool
  run inline RSMI_PRESENT_COPY=inline
  run nt RSMI_PRESENT_COPY=nt
done
for f in $O/*.trace; do echo "$f: $(grep -h 'median' $f | grep -v RSMI | sed 's/ over 1000 calls.*//') $(grep -h 'copy_present' $f) $(grep -h '^cpu ' $f)"; done
for rep in 1 2; do
  for mode in pool inline nt; do
    RSMI_PRESENT_COPY=$mode timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_${mode}_$rep.json 2> $O/c1_${mode}_$rep.err || { tail $O/c1_${mode}_$rep.err; exit 3; }
    echo "$mode $rep $(python3 -c "import json; d=json.load(open('$O/c1_${mode}_$rep.json')); print(d['codec']['decode4_ms'], d['cpu_1t']['avx2_1t']['decode4_ms'], d['gpu_vs_1core'])")"
  done
done
RSMI_PRESENT_COPY=nt timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mailbox.py tests/test_plugin.py -m gpu -x -q -k "decode or Decode or mailbox" --timeout 300 --timeout-method thread > $O/pytest_nt.log 2>&1 || { tail -30 $O/pytest_nt.log; exit 4; }
tail -1 $O/pytest_nt.log
