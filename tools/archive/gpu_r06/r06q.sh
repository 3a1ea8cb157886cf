#!/bin/bash
# r06q: does the calling thread's NUMA node decide the single-message
# latency?  Topology, then config-1 decode / encode pinned to one CPU of
# each NUMA node the job may use, and unpinned (reporting where it ran).
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
python3 tools/numa_probe.py > $O/topology.json || exit 1
cat $O/topology.json
PICK=$(python3 tools/numa_probe.py --pick)
echo "pick: $PICK"
for rep in 1 2; do
  for cpu in $PICK; do
    for W in decode encode; do
      RSMI_PIN_CPU=$cpu RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_cpu${cpu}_$rep.trace 2>&1 || { tail $O/${W}_cpu${cpu}_$rep.trace; exit 2; }
    done
  done
  for W in decode encode; do
    RSMI_TRACE=1 timeout -k 10 120 python3 tools/trace_single.py $W 1000 > $O/${W}_free_$rep.trace 2>&1 || { tail $O/${W}_free_$rep.trace; exit 2; }
  done
done
for f in $O/*.trace; do echo "$f: $(grep -h 'median' $f | grep -v RSMI | sed 's/ over 1000 calls.*//') $(grep -h '^cpu ' $f)"; done
