#!/bin/bash
# Round 2 (o): config-3 erasure cases on the headline workload, and the
# default bench line with the pattern-preparation cost.
set -euo pipefail
O=gpurun_out/r02o
mkdir -p $O
B="python3 bench.py --steps 10 --warmup 3"
timeout -k 10 300 $B > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 240 $B --mode reconstruct --cpu-seconds 0 > $O/rec_random_1_4.json 2> $O/rec.err
timeout -k 10 240 $B --mode reconstruct --cpu-seconds 0 --erase 0,1,2,3 > $O/rec_data_0_1_2_3.json 2>> $O/rec.err
timeout -k 10 240 $B --mode reconstruct --cpu-seconds 0 --erase 6,7,8,9 > $O/rec_data_6_7_8_9.json 2>> $O/rec.err
timeout -k 10 240 $B --mode reconstruct --cpu-seconds 0 --erase 10,11,12,13 > $O/rec_parity_only.json 2>> $O/rec.err
timeout -k 10 240 $B --mode reconstruct --cpu-seconds 0 --erase 3 > $O/rec_one_data.json 2>> $O/rec.err
echo done
