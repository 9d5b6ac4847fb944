#!/bin/bash
# Round 5 call: in-call engine A/B (tools/gpu_ab_pair.sh) and an
# instruction-cache PMC pass of engine_kernel on hotspot (new build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=${A:-abso/base.so} B=${B:-abso/divs.so} TAG=${TAG:-ab2} REPS=${REPS:-2} APPS="${APPS:-bfs streamcluster hotspot heartwall backprop}" \
  bash tools/gpu_ab_pair.sh || exit $?
mkdir -p gpurun_out/pmc_icache
export ASIM_GPU_PROFILE=0
ASIM_NATIVE_SO=${B:-abso/divs.so} timeout -s KILL 90 rocprofv3 --kernel-trace --stats \
  --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS \
  -d gpurun_out/pmc_icache/hotspot -o pmc -- python3 tools/profile_engine.py --app hotspot \
  > gpurun_out/pmc_icache/hotspot.log 2>&1
rc=$?
tail -3 gpurun_out/pmc_icache/hotspot.log
db=$(find gpurun_out/pmc_icache/hotspot -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/pmc_summary.py "$db" engine_kernel
exit $rc
