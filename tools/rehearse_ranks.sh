set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench_nccl1.log 2>&1 || { tail -20 gpurun_out/bench_nccl1.log; exit 1; }
grep '^{' gpurun_out/bench_nccl1.log | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo > gpurun_out/bench_gloo2.log 2>&1 || { tail -20 gpurun_out/bench_gloo2.log; exit 1; }
grep '^{' gpurun_out/bench_gloo2.log | cut -c1-400
