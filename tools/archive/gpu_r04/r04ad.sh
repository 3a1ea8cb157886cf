#!/bin/bash
# Small reconstruct batches read their descriptors in place from pinned
# staging (no copy-engine upload; RSMI_DESC_DIRECT_MAX, default 256 stripes):
# GPU suite, device-stripe fuzz, latency sweep against the upload path
# (RSMI_DESC_DIRECT_MAX=0), default line.
set -o pipefail
O=gpurun_out/r04ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python3 -u tools/fuzz_stripes.py --seconds 90 --seed 777 > $O/fuzz_stripes.json 2> $O/fuzz.err || { cat $O/fuzz_stripes.json; tail -20 $O/fuzz.err; exit 2; }
cat $O/fuzz_stripes.json
for code in "64 80 65536" "10 14 1048576"; do
  set -- $code
  timeout -k 10 200 python3 tools/bench_latency_sweep.py --k $1 --n $2 --shard $3 > $O/sweep_direct_$1.json 2>> $O/sweep.err || exit 3
  RSMI_DESC_DIRECT_MAX=0 timeout -k 10 200 python3 tools/bench_latency_sweep.py --k $1 --n $2 --shard $3 > $O/sweep_upload_$1.json 2>> $O/sweep.err || exit 4
done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
python3 - <<'PY'
import json
O = "gpurun_out/r04ad"
for c in ("64", "10"):
    a = json.load(open(f"{O}/sweep_direct_{c}.json")); b = json.load(open(f"{O}/sweep_upload_{c}.json"))
    for ra, rb in zip(a["rows"], b["rows"]):
        if ra["stripes"] in (1, 4, 16, 64, 256, 512, 16384):
            print(a["code"], ra["stripes"], "rec cached", rb["reconstruct_cached_ms"], "->", ra["reconstruct_cached_ms"], "| new", rb["reconstruct_new_patterns_ms"], "->", ra["reconstruct_new_patterns_ms"])
d = json.load(open(f"{O}/bench.json")); print("line", d["value"], d["roofline"]["frac"], d["breakdown"]["reconstruct_ms"], d["config5"]["reconstruct"]["ms"])
PY
echo done
