#!/bin/bash
# torchrun rehearsals of bench.py on one GPU box: world 2 over gloo (both
# ranks on the one GPU: the multi-rank path, all-gather included) and world 1
# over RCCL (the nccl backend the round-end scaling run uses).
set -o pipefail
mkdir -p gpurun_out
run() {  # run <log> <nproc> <port> <args...>
  local log=$1 np=$2 port=$3; shift 3
  echo "== world $np $*"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$np" --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus "$np" "$@" > "gpurun_out/$log" 2>&1 || exit $?
  grep '^{' "gpurun_out/$log" | tail -n 1 > "gpurun_out/${log%.log}.json"
  grep -o '"value": [0-9.]*\|"parallelism": "[^"]*"' "gpurun_out/${log%.log}.json"
}
run tr_gloo2.log 2 29531 --steps 2 --warmup 1 --backend gloo --no-cpu-baseline --pmc off
run tr_rccl1.log 1 29532 --steps 2 --warmup 1 --no-cpu-baseline --pmc off
