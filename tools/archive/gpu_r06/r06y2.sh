#!/bin/bash
# r06y2: the config-1 leg inside the full default line vs alone, same box.
set -o pipefail
O=gpurun_out/r06y2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/config1_leg.py 50 > $O/c1_alone_1.json 2> $O/c1_alone_1.err || exit 1
timeout -k 10 600 python3 bench.py > $O/bench_1.json 2> $O/bench_1.err || exit 2
timeout -k 10 300 python3 tools/config1_leg.py 50 > $O/c1_alone_2.json 2> $O/c1_alone_2.err || exit 1
timeout -k 10 600 python3 bench.py > $O/bench_2.json 2> $O/bench_2.err || exit 2
for f in $O/c1_alone_1.json $O/c1_alone_2.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['codec']['encode_ms'], d['codec']['decode4_ms'], d['codec']['decode4_arena_ms'], d['gpu_vs_1core'])"; done
for f in $O/bench_1.json $O/bench_2.json; do python3 -c "import json; d=json.load(open('$f'))['config1']; print('$f', d['codec']['encode_ms'], d['codec']['decode4_ms'], d['codec']['decode4_arena_ms'], d['gpu_vs_1core'])"; done
