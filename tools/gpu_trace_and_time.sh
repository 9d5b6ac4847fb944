#!/bin/bash
# On the MI355X box: capture automatic ISA traces of the HIP app suite through
# the instrumented twins (bin/isatrace/<app>), and time + count the plain
# builds under rocprofv3 (4 timing runs each, one pass per counter group).
# Every GPU step has its own time limit and the script stops at the first
# failure.  SUITE selects the app list (define-all-apps.yml).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
SUITE=${SUITE:-rodinia_2.0-ft-hip}
out=$R/gpurun_out/corr
mkdir -p $out
timeout -k 10 900 python $R/accel_sim_framework_distributed_amd/hw_stats/run_hw_trace.py -B $SUITE -b \
  -o $out/traces > $out/trace.log 2>&1 || { echo "tracing failed"; tail -20 $out/trace.log; exit 1; }
timeout -k 10 900 python $R/accel_sim_framework_distributed_amd/hw_stats/run_hw.py -B $SUITE -R 4 \
  --counter_groups -o $out/hw > $out/hw.log 2>&1 || { echo "hw timing failed"; tail -20 $out/hw.log; exit 1; }
du -sh $out/traces $out/hw
grep -h PASSED -c $out/trace.log
