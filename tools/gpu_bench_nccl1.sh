#!/bin/bash
# Bench on one MI355X, then the same bench as a 1-rank torchrun job on the
# nccl (RCCL) backend: the path the driver's multi-GPU scaling run takes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py > gpurun_out/bench_r2e.log 2>&1
timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 2 --warmup 1 --dist-backend nccl > gpurun_out/bench_nccl1_r2e.log 2>&1
