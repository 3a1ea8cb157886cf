#!/bin/bash
# Longer randomised fuzzing of the final round-5 engine (new seeds): the
# host API incl. encode/decode batches, and device stripes.
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 330 python3 tools/fuzz_host_api.py --seconds 280 --seed 17 > $O/fuzz_host.json 2> $O/fuzz_host.err || { tail -5 $O/fuzz_host.err; cat $O/fuzz_host.json; exit 1; }
cat $O/fuzz_host.json
timeout -k 10 330 python3 tools/fuzz_stripes.py --seconds 280 --seed 17 > $O/fuzz_stripes.json 2> $O/fuzz_stripes.err || { tail -5 $O/fuzz_stripes.err; cat $O/fuzz_stripes.json; exit 2; }
cat $O/fuzz_stripes.json
