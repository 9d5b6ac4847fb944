#!/bin/bash
# The correlation pipeline of tools/gpu_correlate.sh, steps 2-3, on this host
# with the CPU engine: re-simulates the traces a GPU run archived
# (gpurun_out/corr/trace_tgz) with a config directory and correlates every
# statistic against that run's rocprofv3 counters (gpurun_out/corr/hw).
#   tools/local_full_correlate.sh [out_dir]
# (the suite's MI355X_TUNED config reads configs/tuned/AMD_Instinct_MI355X:
# edit that directory to try a change)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
out=${1:-/tmp/lcorr}
src=${CORR_SRC:-$R/gpurun_out/corr}
rm -rf $out && mkdir -p $out/traces
for t in $src/trace_tgz/*.tgz; do tar xzf $t -C $out/traces; done
export PROCMAN_STATE=$out/procman.json ASIM_JOB_LOGDIR=$out/logs
JL=$R/util/job_launching
python $JL/run_simulations.py -B ${SUITE:-rodinia_2.0-ft-hip} -C ${CFG:-MI355X_TUNED} -T $out/traces -N lcorr -l local \
  -r $out/simrun -c ${JOBS:-8} --threads 1 > $out/launch.log 2>&1 || { echo "launch failed"; tail $out/launch.log; exit 1; }
python $JL/monitor_func_test.py -N lcorr -r $out/simrun -S 5 -T 1200 -K -j procman > $out/monitor.log 2>&1
tail -3 $out/monitor.log
python $JL/get_stats.py -N lcorr -r $out/simrun -k -K -I > $out/stats_per_kernel.csv
python $JL/get_stats.py -N lcorr -r $out/simrun -I > $out/stats.csv
python $R/util/plotting/plot-correlation.py -c $out/stats_per_kernel.csv -H $src/hw -B 1 --clock_mhz 2400 \
  -p mi355x -o $out/correl | grep -v "^wrote" | tee $out/correl.log
