#!/bin/bash
# Syndrome-solve micro-benchmark: split-table MAC vs bit-plane combinations
# in LDS (tools/ubench/solve_lds_ubench.hip).
set -o pipefail
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 120 tools/ubench/build/solve_lds_ubench > $O/solve_lds.log 2>&1 || exit 1
timeout -k 10 120 tools/ubench/build/solve_lds_ubench >> $O/solve_lds.log 2>&1 || exit 2
echo done
