#!/bin/bash
# Round 5 power validation on one MI355X: fresh amd-smi measurement of the
# 58-kernel suite, the kernels' durations at the traced sizes, fresh ISA
# traces (archived for local re-fits), and the held-out fit with the tuned
# config as committed (-sim_single_valu 1, fitted L1 / LDS data paths).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/power_r5
mkdir -p $out
cd /tmp
timeout -k 10 300 $R/bin/apps/power_suite measure 1.5 > $out/measured.csv 2> $out/measure.err \
  || { echo "measure failed"; tail $out/measure.err; exit 1; }
timeout -k 10 120 $R/bin/apps/power_suite time > $out/durations.csv 2> $out/durations.err \
  || { echo "time failed"; tail $out/durations.err; exit 1; }
rm -rf /tmp/pwr_traces
ASIM_TRACE_DIR=/tmp/pwr_traces timeout -k 10 300 $R/bin/isatrace/power_suite trace > $out/trace.log 2>&1 \
  || { echo "trace failed"; tail $out/trace.log; exit 1; }
tail -1 $out/trace.log
du -sh /tmp/pwr_traces
tar czf $out/pwr_traces.tgz -C /tmp pwr_traces
sz=$(du -m $out/pwr_traces.tgz | cut -f1); [ "$sz" -gt 40 ] && rm -f $out/pwr_traces.tgz && echo "trace archive too big ($sz MB)"
timeout -k 10 800 python3 $R/accel_sim_framework_distributed_amd/power/mi355x_validation.py -t /tmp/pwr_traces/kernelslist.g \
  -m $out/measured.csv -c $R/configs/tuned/AMD_Instinct_MI355X -e cpu-split -w /tmp/pwr_work \
  -j $out/validation.json -o $out/accelwattch_sass_sim_calibrated.xml --heldout > $out/validation.log 2>&1; e=$?
tail -32 $out/validation.log
rm -rf /tmp/pwr_traces /tmp/pwr_work
exit $e
