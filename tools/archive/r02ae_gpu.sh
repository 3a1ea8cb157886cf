#!/bin/bash
# r02ae: GPR-indexed bit-plane syndrome solve (s_set_gpr_idx_on + v_xor_b32)
# vs the split-table solve.  v2: s_nop 1 after every index write (correct);
# v4: s_nop 0 (probe).  Correctness first (tools/diag/diag_gpr.py), then
# config-5 reconstruct timings, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02ae
mkdir -p $O
L=$R/noise-erasurecode-plugin_amd/lib_ab
RSMI_LIB=$L/v4/librsmi.so timeout -k 10 100 python3 tools/diag/diag_gpr.py quick 2>&1 | grep -v "amdgpu.ids\|  stripe" > $O/diag_v4.txt || exit 1
run() { timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --mode reconstruct "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['reconstruct_GBps'], b['reconstruct_ms'])"; }
C="--k 64 --n 80 --shard 65536 --stripes 16384"
for rep in 1 2; do
  for lib in v2 v4 split; do
    export RSMI_LIB=$L/$lib/librsmi.so
    echo "== $lib rep $rep: e=16 fresh" >> $O/ab.log; run $C --emin 16 --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== $lib rep $rep: e=1..16 fresh" >> $O/ab.log; run $C --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 3
  done
done
echo ok
