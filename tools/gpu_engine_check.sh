#!/bin/bash
# GPU engine check after an engine change: bit-exact GPU tests, per-app
# engine wall times with the stage profiler (bfs, hotspot), then the bench.
# usage (on the GPU box): bash tools/gpu_engine_check.sh  -> gpurun_out/chk_*.log
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk_gputest.log 2>&1
for app in bfs hotspot streamcluster nw; do
  timeout -k 10 120 python3 tools/profile_engine.py --app $app > gpurun_out/chk_stage_$app.log 2>&1
done
timeout -k 10 420 python -u bench.py > gpurun_out/chk_bench.log 2>&1
