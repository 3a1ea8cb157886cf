#!/bin/bash
# Round-5 final tree: N = 8 and N = 4 gloo rehearsals of the bench line (ranks sharing the one
# GPU, gather leg verified over two steps) on the final tree, then smoke().
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
RSMI_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 8 --stripes 128 --shard 262144 --steps 3 --warmup 1 --cpu-seconds 1 --gather-stripes 32 --gather-timeout 240 > $O/gpus8_gloo.json 2> $O/gpus8_gloo.err || { echo "N=8 rc=$?"; tail -20 $O/gpus8_gloo.err; exit 1; }
RSMI_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 4 --stripes 256 --shard 1048576 --steps 3 --warmup 1 --cpu-seconds 1 --gather-stripes 64 --gather-timeout 240 > $O/gpus4_gloo.json 2> $O/gpus4_gloo.err || { echo "N=4 rc=$?"; tail -20 $O/gpus4_gloo.err; exit 2; }
for f in gpus8_gloo gpus4_gloo; do python3 -c "
import json; d=json.load(open('$O/$f.json')); g=d['gather']
print('$f', d['n_gpus'], d['value'], [r['bytes'] for r in d['per_rank']], g['status'], g['backend'], g.get('chunks'), g.get('verified'))"; done
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
tail -1 $O/smoke.log
echo done
