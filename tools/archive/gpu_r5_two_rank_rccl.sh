#!/bin/bash
# Round 5: multi-rank rehearsal of bench.py on one MI355X: two ranks (both on
# the one GPU), RCCL collectives, node placement per rank, rank-0 plan.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 $R/bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend nccl > $R/gpurun_out/bench_2rank_rccl.log 2>&1
e=$?
grep '^{"metric"' $R/gpurun_out/bench_2rank_rccl.log | cut -c1-600
tail -3 $R/gpurun_out/bench_2rank_rccl.log
exit $e
