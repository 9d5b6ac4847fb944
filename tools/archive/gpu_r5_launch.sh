#!/bin/bash
# Round 5: what a kernel's rocprofv3 duration holds when it is queued behind
# another kernel, chained, launched after a host gap or after a copy
# (bin/ubench/ub_launch_seq, device-clock stamps of every launch's execution
# window; accel_sim_framework_distributed_amd/hw_stats/launch_seq.py), and the
# power suite's kernel durations at the measured (steady-state) sizes.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/launch_seq
mkdir -p $out
timeout -k 10 200 python3 $R/accel_sim_framework_distributed_amd/hw_stats/launch_seq.py -o $out --exe $R/bin/ubench/ub_launch_seq \
  -j $out/launch_seq.json > $out/summary.txt 2>&1; e=$?
cat $out/summary.txt | tail -40
[ $e -eq 0 ] || exit $e
# the power suite's kernels at the measured sizes (steady-state durations)
cd /tmp && timeout -k 10 120 $R/bin/apps/power_suite time_full > $out/power_suite_time_full.csv 2> $out/power_suite_time_full.err
e=$?; tail -3 $out/power_suite_time_full.csv; [ $e -eq 0 ] || exit $e
# binary-only traced nw == source-built traced nw (GPU test tier subset)
cd $R && timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_isatrace.py -k "binary_path" > $out/pytest_binary_path.log 2>&1; e=$?; tail -3 $out/pytest_binary_path.log; exit $e
