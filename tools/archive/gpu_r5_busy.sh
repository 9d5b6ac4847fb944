#!/bin/bash
# Round 5: per-kernel busy cycles of the HIP Rodinia suite (GRBM_GUI_ACTIVE
# over GRBM_COUNT, SQ_BUSY_CYCLES over SQ_CYCLES): how much of each kernel's
# rocprofv3 duration is execution and how much is launch / completion
# overhead -- the split the simulator's launch model needs.  One counter pass
# per app (rocprofv3 --pmc, kernel dispatches serialised), 2 timing runs.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/busy
mkdir -p $out
timeout -k 10 600 python3 $R/accel_sim_framework_distributed_amd/hw_stats/run_hw.py -B rodinia_2.0-ft-hip -R 2 \
  -c "GRBM_COUNT,GRBM_GUI_ACTIVE,SQ_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES" -o $out/hw > $out/hw.log 2>&1; e=$?
tail -3 $out/hw.log
du -sh $out
exit $e
