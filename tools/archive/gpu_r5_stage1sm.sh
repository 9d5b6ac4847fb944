#!/bin/bash
# Stage profile of the one-SM engine (profiling build of engine_kernel) and
# the loopback exchange cost record.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5_stage
mkdir -p $o
for app in hotspot bfs; do
  ASIM_GPU_PROFILE=1 timeout -k 10 180 python3 tools/engine_pmc_1sm.py --app $app > $o/stage_$app.log 2>&1 || exit $?
  grep -v amdgpu.ids $o/stage_$app.log | head -60
done
timeout -k 10 300 python3 tools/rccl_epoch_cost.py --iters 1000 --out $o/rccl_loopback_epoch_cost.json > $o/rccl.log 2>&1
rc=$?
tail -3 $o/rccl.log
exit $rc
