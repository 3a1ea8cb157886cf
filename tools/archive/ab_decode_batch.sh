# GPU parity, then receive batching (rs_decode_batch) with chunked staging /
# PCIe overlap vs the build before (lib_ab/base: one staging copy, one H2D,
# one D2H), interleaved runs on one box.
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
OLD=$GRAFT_REPO_ROOT/noise-erasurecode-plugin_amd/lib_ab/base/librsmi.so
for r in 1 2 3 4 5; do
  echo "new"; timeout -k 10 300 python3 tools/bench_host_api.py --batch-only --batch-reps 10 || exit 1
  echo "old"; RSMI_LIB=$OLD timeout -k 10 300 python3 tools/bench_host_api.py --batch-only --batch-reps 10 || exit 1
done
