#!/bin/bash
# PC sampling of the engine kernel on one app (instruction-level stall view).
set -e
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pcs
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1 || true
grep -i -A3 "pc.sampl\|PC_SAMPLING\|stochastic\|host_trap" gpurun_out/pcs/list.txt | head -40 || true
ASIM_GPU_PROFILE=0 timeout -k 10 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-host_trap} \
  --pc-sampling-unit ${UNIT:-time} --pc-sampling-interval ${IVAL:-1} -d gpurun_out/pcs/out -o pcs --output-format csv \
  -- python3 tools/profile_engine.py --app ${APP:-bfs} > gpurun_out/pcs/run.log 2>&1
find gpurun_out/pcs -name "*.csv" | head
