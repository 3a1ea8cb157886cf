#!/bin/bash
# Decode latency build (descriptor word as an argument, identity survivor ids,
# strided staging, cached staging aliases) with call arrays bound once in
# the probe and the config1 leg: GPU suite, latency probe x3, default line.
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 2; }
done
for f in $O/probe_*.json; do echo "$f $(cat $f)"; done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['breakdown']['encode_ms'], d['breakdown']['reconstruct_ms'], json.dumps(d['config1']['codec']), json.dumps(d['config1']['cpu_1t']['avx2_1t']), d['config5']['encode']['ms'], d['config5']['reconstruct']['ms'])"
echo done
