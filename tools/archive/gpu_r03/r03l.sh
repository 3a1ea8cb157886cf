#!/bin/bash
# After the sign-extension fix: the -M diagnostic build over the bit-sliced
# reconstruct tests must print no mask disagreement; then r03j (GPU suite,
# smoke, mask-record A/B against lib_ab/prev).
set -o pipefail
O=gpurun_out/r03l
mkdir -p $O
RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/dbg/librsmi.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_parity.py -x -v -s -m gpu --timeout 120 --timeout-method thread -k "null_stream or bitslice or row_subset or xcd or ptrs" > $O/dbg_tests.txt 2>&1 || exit 1
if grep -q RSMI_MASK_MISMATCH $O/dbg_tests.txt; then echo "mask mismatch"; exit 2; fi
bash tools/gpu/r03j.sh || exit 3
echo done
