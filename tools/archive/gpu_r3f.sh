#!/bin/bash
# Round-3 experiment: GPU-engine suite throughput against the blocks per
# simulation (ASIM_GPU_BLOCKS caps a simulation's workgroups; its SMs and
# memory channels then time-slice over them, so more simulations share the
# 256 CUs at once), then the node bench with the same caps.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3f
mkdir -p $out
cd $R
for b in 0 56 37 28; do
  ASIM_GPU_BLOCKS=$b timeout -k 10 300 python bench.py --engine gpu > $out/bench_gpu_b$b.log 2>&1
  echo "blocks=$b $(tail -1 $out/bench_gpu_b$b.log | cut -c1-160)"
done
for b in 37; do
  ASIM_GPU_BLOCKS=$b timeout -k 10 300 python bench.py > $out/bench_node_b$b.log 2>&1
  echo "node blocks=$b $(tail -1 $out/bench_node_b$b.log | cut -c1-160)"
done
