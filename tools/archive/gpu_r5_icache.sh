#!/bin/bash
# Round 5: is the instruction cache cold at every kernel launch?  Four
# launches of the same kernel under rocprofv3 SQC counters (ub_icache_launch).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/ubench/icache_launch
mkdir -p $out
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $out -o run \
  -- $R/bin/ubench/ub_icache_launch > $out/run.log 2>&1; e=$?
tail -2 $out/run.log
[ $e -eq 0 ] || exit $e
python3 $R/accel_sim_framework_distributed_amd/hw_stats/icache_launch.py $out > $R/gpurun_out/ubench/ub_icache_launch.log
cat $R/gpurun_out/ubench/ub_icache_launch.log
