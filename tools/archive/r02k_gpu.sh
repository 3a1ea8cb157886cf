# r02k: rehearsal of the driver's multi-rank bench on ONE GPU with gloo
# (2 and 4 ranks sharing the device; the driver runs RCCL, one rank per GPU):
# local placement (the scaling line) and sharded placement (RCCL gather path,
# staged through host under gloo).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02k
mkdir -p $O
export RSMI_BENCH_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 $R/bench.py --gpus 2 --steps 3 --warmup 1 --stripes 3000 > $O/local_n2.json 2> $O/local_n2.err || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29522 $R/bench.py --gpus 4 --steps 3 --warmup 1 --stripes 1000 > $O/local_n4.json 2> $O/local_n4.err || exit 2
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 $R/bench.py --placement sharded --gpus 2 --steps 2 --warmup 1 --stripes 64 --shard 65536 > $O/sharded_n2.json 2> $O/sharded_n2.err || exit 3
echo ok
