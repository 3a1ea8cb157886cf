#!/bin/bash
# Final robustness evidence of HEAD: a 5-minute randomised soak of every kernel
# family and a 150 s 8-thread concurrency soak with pattern-cache evictions.
set -o pipefail
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 400 python3 -u tools/fuzz_stripes.py --seconds 300 --seed 123 > $O/fuzz.json 2> $O/fuzz.err || exit 1
RSMI_PATTERN_CAP=2000 timeout -k 10 240 python3 -u tools/soak_concurrency.py --seconds 150 --threads 8 > $O/soak.json 2> $O/soak.err || exit 2
echo done
