#!/bin/bash
# r06b: the bit-plane solve of the syndrome reconstruct -- parity tests of the
# bit-sliced kernels, then a same-box A/B against the round-5 split-table
# solve (lib_ab/splitsolve, gen_bitslice -s) on the config-5 shapes.
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_set.py -m gpu -x -v \
  -k "(bitslice or config5 or reconstruct or rebuild or set00) and not mask_diagnostic" \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_TAG=r06b AB_LIBS="cur splitsolve" AB_REPS=2 timeout -k 10 900 bash tools/ab_libs.sh || { echo "ab failed"; tail $O/ab.err; exit 2; }
cat $O/ab.log
