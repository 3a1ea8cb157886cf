#!/bin/bash
# r06r: single-message chunk splits with the caller on the GPU's NUMA node
# (as bench.py now runs): "33" (two chunks), "20,60", "25,60", "15,50" (three);
# then the config-1 leg alone, pinned, twice; mailbox tests under "20,60".
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" RSMI_PIN_GPU_NUMA=1 RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_${name}_$rep.trace 2>&1 || { tail $O/${W}_${name}_$rep.trace; exit 2; }
}
for rep in 1 2; do
  for W in decode encode; do
    run s33 RSMI_CHUNK_SPLIT=33
    run s20_60 RSMI_CHUNK_SPLIT=20,60
    run s25_60 RSMI_CHUNK_SPLIT=25,60
    run s15_50 RSMI_CHUNK_SPLIT=15,50
  done
done
for f in $O/*.trace; do echo "$f: $(grep -h 'median' $f | grep -v RSMI | sed 's/ over 1000 calls.*//') $(grep -h '^cpu ' $f)"; done
grep -h "^affinity" $O/decode_s33_1.trace
RSMI_CHUNK_SPLIT=20,60 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mailbox.py tests/test_gpu_parity.py -m gpu -x -q -k "mailbox or decode or encode" --timeout 300 --timeout-method thread > $O/pytest_split.log 2>&1 || { tail -40 $O/pytest_split.log; exit 3; }
tail -1 $O/pytest_split.log
for rep in 1 2; do
  timeout -k 10 300 python3 tools/config1_leg.py 200 > $O/c1_$rep.json 2> $O/c1_$rep.err || { tail $O/c1_$rep.err; exit 4; }
  cat $O/c1_$rep.json
done
