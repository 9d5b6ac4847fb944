#!/bin/bash
# PMC pass over one suite app on the (non-profiling) GPU engine.
# usage: APP=hotspot bash tools/gpu_pmc.sh  -> gpurun_out/pmc_<app>/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
APP=${APP:-hotspot}
mkdir -p gpurun_out
export ASIM_GPU_PROFILE=0
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmc_$APP -o pmc -- python3 tools/profile_engine.py --app $APP > gpurun_out/pmc_$APP.log 2>&1
