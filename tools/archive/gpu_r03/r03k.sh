#!/bin/bash
# Diagnostic: the mask-record reconstruct built with -M (lib_ab/dbg) codes
# with the id-row masks and prints any disagreement with the host record.
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
RSMI_LIB=$PWD/noise-erasurecode-plugin_amd/lib_ab/dbg/librsmi.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_concurrency.py -x -v -s -m gpu --timeout 120 --timeout-method thread -k "null_stream or concurrent_decode" > $O/dbg_tests.txt 2>&1 || exit 1
echo done
