#!/bin/bash
# Round-4 engine profile on the current tree: stage profile + two SQ PMC
# passes of engine_kernel on bfs and hotspot, and a stochastic PC-sampling
# attempt (instruction-level view of the critical block).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4prof${TAG:+_$TAG}
mkdir -p $OUT
for app in ${APPS:-bfs hotspot}; do
  timeout -k 10 150 python3 tools/profile_engine.py --app $app > $OUT/stage_$app.log 2>&1
  ASIM_GPU_PROFILE=0 timeout -k 10 150 python3 tools/profile_engine.py --app $app > $OUT/plain_$app.log 2>&1
  if [ -z "$NOPMC" ]; then
  export ASIM_GPU_PROFILE=0
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc1_$app -o pmc -- python3 tools/profile_engine.py --app $app > $OUT/pmc1_$app.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $OUT/pmc2_$app -o pmc -- python3 tools/profile_engine.py --app $app > $OUT/pmc2_$app.log 2>&1
  unset ASIM_GPU_PROFILE
  fi
done
if [ -n "$PCS" ]; then
  ASIM_GPU_PROFILE=0 timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
    --pc-sampling-unit cycles --pc-sampling-interval ${IVAL:-65536} -d $OUT/pcs -o pcs --output-format csv \
    -- python3 tools/profile_engine.py --app bfs > $OUT/pcs_run.log 2>&1 || echo "pc sampling failed rc=$?"
fi
echo done
