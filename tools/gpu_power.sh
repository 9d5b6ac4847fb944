#!/bin/bash
# On the MI355X box: AccelWattch validation on the 24-kernel power suite.
# Measure socket power of every kernel (bin/apps/power_suite measure), capture
# automatic ISA traces of the same kernels (bin/isatrace/power_suite trace),
# simulate them with the tuned MI355X config + power model, fit the grouped
# scaling factors and report in-sample and leave-one-out MAPE.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${PWR_OUT:-power}
mkdir -p $out
cd /tmp
timeout -k 10 300 $R/bin/apps/power_suite measure ${PWR_SECS:-1.5} > $out/measured.csv 2> $out/measure.err \
  || { echo "measure failed"; tail $out/measure.err; exit 1; }
cat $out/measured.csv
rm -rf /tmp/pwr_traces
ASIM_TRACE_DIR=/tmp/pwr_traces timeout -k 10 300 $R/bin/isatrace/power_suite trace > $out/trace.log 2>&1 \
  || { echo "trace failed"; tail $out/trace.log; exit 1; }
tail -1 $out/trace.log
du -sh /tmp/pwr_traces
# cpu-split: every kernel is its own CPU-engine simulation, one per host core
timeout -k 10 ${PWR_SIM_SECS:-800} python3 $R/accel_sim_framework_distributed_amd/power/mi355x_validation.py -t /tmp/pwr_traces/kernelslist.g \
  -m $out/measured.csv -c $R/configs/tuned/AMD_Instinct_MI355X -e ${PWR_ENGINE:-cpu-split} -w /tmp/pwr_work \
  -j $out/validation.json -o $out/accelwattch_sass_sim_calibrated.xml ${PWR_HELDOUT:+--heldout} > $out/validation.log 2>&1; e=$?
cat $out/validation.log | tail -32
rm -rf /tmp/pwr_traces /tmp/pwr_work
exit $e
