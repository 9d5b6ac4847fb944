#!/bin/bash
# Round 5, call 1: baseline GPU-engine times per app (profiler off) and
# host-trap PC sampling of engine_kernel on bfs (instruction-level hot spots).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5pcs
export ASIM_GPU_PROFILE=0
for app in bfs streamcluster hotspot; do
  timeout -k 10 120 python3 tools/profile_engine.py --app $app >> gpurun_out/r5pcs/base_times.log 2>&1 || exit $?
done
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
  --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/r5pcs/out -o pcs --output-format csv \
  -- python3 tools/profile_engine.py --app bfs > gpurun_out/r5pcs/run.log 2>&1
rc=$?
find gpurun_out/r5pcs -name "*.csv" | head
exit $rc
