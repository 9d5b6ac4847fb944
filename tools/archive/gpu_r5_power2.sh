#!/bin/bash
# Round 5, power refit with the issue-weighted static column (STATIC_ISSUEP):
# fresh ISA traces of the 58-kernel suite, simulated with the tuned config,
# fitted against the round-5 measurement (profiles/r5/power_measured_r5.csv:
# the measured power does not depend on the model) -- calibration on the 30
# single-unit kernels, validation on the 28 held-out mixes.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${POWER_OUT:-power_r5b}
mkdir -p $out
cd /tmp
rm -rf /tmp/pwr_traces
ASIM_TRACE_DIR=/tmp/pwr_traces timeout -k 10 300 $R/bin/isatrace/power_suite trace > $out/trace.log 2>&1 \
  || { echo "trace failed"; tail $out/trace.log; exit 1; }
tail -1 $out/trace.log
timeout -k 10 800 python3 $R/accel_sim_framework_distributed_amd/power/mi355x_validation.py -t /tmp/pwr_traces/kernelslist.g \
  -m $R/profiles/r5/power_measured_r5.csv -c $R/configs/tuned/AMD_Instinct_MI355X -e cpu-split -w /tmp/pwr_work \
  -j $out/validation.json -o $out/accelwattch_sass_sim_calibrated.xml --heldout > $out/validation.log 2>&1; e=$?
tail -6 $out/validation.log
rm -rf /tmp/pwr_traces /tmp/pwr_work
exit $e
