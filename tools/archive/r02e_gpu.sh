# r02e: GPU suite, then the headline + config-5 benches on the current build
# and on the round-1 build (lib_ab/r01, RSMI_LIB) interleaved, then the
# sharded placement under torchrun (world 1).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
run() { timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown']; print(d['value'], b['encode_GBps'], b['reconstruct_GBps'], b['encode_ms'], b['reconstruct_ms'], d['roofline']['frac'])"; }
for rep in 1 2; do
  for lib in cur r01; do
    if [ $lib = r01 ]; then export RSMI_LIB=$R/noise-erasurecode-plugin_amd/lib_ab/r01/librsmi.so; else unset RSMI_LIB; fi
    echo "== $lib rep $rep: RS(10,4) default" >> $O/ab.log; run >> $O/ab.log 2>> $O/ab.err || exit 2
    echo "== $lib rep $rep: RS(64,16) e=1..16 fresh" >> $O/ab.log; run --k 64 --n 80 --shard 65536 --stripes 16384 --emax 16 >> $O/ab.log 2>> $O/ab.err || exit 3
  done
done
unset RSMI_LIB
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 $R/bench.py --placement sharded --steps 5 --warmup 2 --cpu-seconds 0 > $O/sharded_world1.json 2> $O/sharded_world1.err || exit 4
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $O/local_world1.json 2> $O/local_world1.err || exit 5
echo ok
