#!/bin/bash
# On the MI355X box: capture
# asim_trace traces of the HIP app suite, and time the plain builds under
# rocprofv3 (4 runs each).  Every GPU step has its own time limit and the
# script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/corr
mkdir -p $out
timeout -k 10 900 python $R/accel_sim_framework_distributed_amd/hw_stats/run_hw_trace.py -B asim_hip_apps -b \
  -o $out/traces > $out/trace.log 2>&1 || { echo "tracing failed"; tail -20 $out/trace.log; exit 1; }
timeout -k 10 900 python $R/accel_sim_framework_distributed_amd/hw_stats/run_hw.py -B asim_hip_apps -R 4 \
  -o $out/hw > $out/hw.log 2>&1 || { echo "hw timing failed"; tail -20 $out/hw.log; exit 1; }
du -sh $out/traces $out/hw
grep -h PASSED -c $out/trace.log
