#!/bin/bash
# One-SM engine diagnostics: wall per simulated SM cycle on both engines and
# two rocprofv3 PMC passes of engine_kernel (instructions and stall shares).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5_1sm
mkdir -p $o
export ASIM_GPU_PROFILE=0
for app in hotspot bfs; do
  for eng in gpu cpu; do
    timeout -k 10 120 python3 tools/engine_pmc_1sm.py --app $app --engine $eng 2>&1 | grep -v amdgpu.ids >> $o/times.log || exit $?
  done
done
cat $o/times.log
p=1
for cs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS" \
          "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU"; do
  for app in hotspot bfs; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $cs -d $o/pmc${p}_$app -o pmc -- \
      python3 tools/engine_pmc_1sm.py --app $app > $o/pmc${p}_$app.log 2>&1 || exit $?
    db=$(find $o/pmc${p}_$app -name "*.db" | head -1)
    python3 tools/pmc_summary.py "$db" engine_kernel > $o/pmc${p}_$app.json
    echo "== pass $p $app"; cat $o/pmc${p}_$app.json
  done
  p=$((p+1))
done
