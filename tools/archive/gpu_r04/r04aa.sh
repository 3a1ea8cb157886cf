#!/bin/bash
# Config-3 worst case (4 data erasures in every stripe) and config 2's
# streamed mode (pinned host memory, PCIe-inclusive) on the final build.
set -o pipefail
O=gpurun_out/r04aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --mode reconstruct --erase 0,1,2,3 --cpu-seconds 0 --no-extra-legs > $O/worst.json 2> $O/worst.err || { tail -20 $O/worst.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/worst.json')); print('worst', d['value'], json.dumps(d['breakdown']))"
timeout -k 10 300 python3 bench.py --mode encode --stream --cpu-seconds 0 --no-extra-legs > $O/stream.json 2> $O/stream.err || { tail -20 $O/stream.err; exit 2; }
python3 -c "import json; d=json.load(open('$O/stream.json')); print('stream', d['value'], d['unit'], json.dumps(d.get('breakdown', {}))[:600])"
echo done
