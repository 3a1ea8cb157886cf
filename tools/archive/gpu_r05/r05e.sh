#!/bin/bash
# Knob A/Bs on the shipped build: RS(10,4) headline reconstruct block order
# (XCD region of 128 / 256 = a stripe (default) / 512 / 1024 blocks),
# temporal cache policy (RSMI_NT=0), address-order descriptors; config-5
# syndrome reconstruct with 2 / 4 stripes per XCD region; and the CPU cost of
# the host API's polled waits under an 8-thread soak (default bounded polling,
# round-4 polling of every wait, no polling).
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
H="--mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 10 --warmup 2"
C5="--k 64 --n 80 --shard 65536 --stripes 16384 --mode reconstruct --cpu-seconds 0 --no-extra-legs --steps 8 --warmup 2"
one() {
  local tag=$1; shift
  timeout -k 10 200 python3 bench.py "$@" 2>> $O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print('$tag', b['reconstruct_ms'], b['reconstruct_GBps'])" >> $O/ab.log
}
for rep in 1 2; do
  one h_default $H || exit 2
  RSMI_XCD_REC_REGION=128 one h_region128 $H || exit 3
  RSMI_XCD_REC_REGION=512 one h_region512 $H || exit 4
  RSMI_XCD_REC_REGION=1024 one h_region1024 $H || exit 5
  RSMI_NT=0 one h_temporal $H || exit 6
  RSMI_NO_SORT=1 one h_nosort $H || exit 7
  one c5_default $C5 || exit 8
  RSMI_XCD_BS_STRIPES=2 one c5_bs2 $C5 || exit 9
  RSMI_XCD_BS_STRIPES=4 one c5_bs4 $C5 || exit 10
done
cat $O/ab.log
S="--seconds 20 --threads 8 --code 10:14 --shard 104858"
RSMI_PATTERN_CAP=2000 timeout -k 10 120 python3 tools/soak_concurrency.py $S > $O/soak_default.json 2>> $O/soak.err || exit 11
RSMI_PATTERN_CAP=2000 RSMI_SYNC_ADAPTIVE=0 timeout -k 10 120 python3 tools/soak_concurrency.py $S > $O/soak_pollall.json 2>> $O/soak.err || exit 12
RSMI_PATTERN_CAP=2000 RSMI_SYNC_SPIN_US=0 timeout -k 10 120 python3 tools/soak_concurrency.py $S > $O/soak_nopoll.json 2>> $O/soak.err || exit 13
cat $O/soak_*.json
echo done
