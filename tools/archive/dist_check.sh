set -o pipefail
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --cpu-seconds 0 || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --steps 3 --warmup 1 --placement sharded --stripes 512 || exit 2
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --placement sharded --stripes 512 || exit 3
