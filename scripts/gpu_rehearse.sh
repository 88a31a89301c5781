set -e
export PYTHONUNBUFFERED=1
timeout -k 10 240 python scripts/ablate.py C3 > gpurun_out/ablate_c3_now.log 2>&1
timeout -k 10 300 python scripts/ablate.py C5B > gpurun_out/ablate_c5b.log 2>&1
NLOSGR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1
NLOSGR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --shard > gpurun_out/bench_gloo2_shard.log 2>&1
