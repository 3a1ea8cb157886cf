#!/bin/bash
# Small messages staged once and coded by one launch (encode_staged /
# decode_staged) + the no-barrier syndrome kernel: GPU suite, latency probe,
# host API table, and the default bench line.
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_$rep.json 2>> $O/probe.err || exit 2
done
RSMI_NO_STAGE_SMALL=1 timeout -k 10 120 python3 tools/probe_latency.py > $O/probe_pipeline.json 2>> $O/probe.err || exit 3
cat $O/probe_*.json
timeout -k 10 300 python3 tools/bench_host_api.py --reps 30 > $O/host_api.json 2> $O/host_api.err || exit 4
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 5
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['config1']['codec']), json.dumps(d['config1']['cpu_1t']['avx2_1t']), d['config5']['encode']['ms'], d['config5']['reconstruct']['ms'])"
echo done
