#!/bin/bash
# RS(10,4) headline encode knobs on the round-5 engine: XCD block order for
# the split-table encode (region = a stripe's 256 blocks, 128, 512), two /
# four column chunks per block (software-pipelined survivor loads), both
# modes; two interleaved reps.
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
H="--mode both --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
one() {
  local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag', b['encode_ms'], b['reconstruct_ms'], b['encode_GBps'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  one default $H || exit 2
  RSMI_XCD_ENC_REGION=256 one enc_xcd256 $H || exit 3
  RSMI_XCD_ENC_REGION=128 one enc_xcd128 $H || exit 4
  RSMI_XCD_ENC_REGION=512 one enc_xcd512 $H || exit 5
  RSMI_ITERS=2 one iters2 $H || exit 6
  RSMI_ITERS=4 one iters4 $H || exit 7
done
cat $O/ab.log
echo done
