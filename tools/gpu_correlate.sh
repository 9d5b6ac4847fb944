#!/bin/bash
# Full MI355X correlation pipeline on the GPU box:
#  0. micro-benchmarks (incl. rocprofv3-fitted launch latency) -> tuner ->
#     configs/tuned/AMD_Instinct_MI355X (copied to gpurun_out/corr/tuned)
#  1. capture automatic ISA traces (isatrace twins) + rocprofv3 timings and
#     counters (tools/gpu_trace_and_time.sh)
#  2. simulate every trace with the tuned MI355X config (run_simulations via the
#     local procman; ENG=GPU (default): the MI355X cycle engine, one job per
#     GPU slot; ENG=CPU: the CPU engine), wait with monitor_func_test
#  3. get_stats (per kernel) + correlator -> cycle MAE vs hardware
# Only the small outputs are kept (traces are archived if they fit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/corr
mkdir -p $out
UBENCH_PROGS="ub_config ub_bw_widths ub_cache_lat ub_cache_policy ub_alu ub_wave_issue ub_lds ub_mfma ub_mfma_shapes ub_icache ub_atomic_kernel ub_launch ub_mem_bw ub_l2_release ub_kernel_lat_tb ub_copy_engine ub_regfile ub_l1_stride ub_mem_lat" \
  bash $R/tools/run_ubench.sh $R/gpurun_out/ubench > $out/ubench.log 2>&1 || { echo "ubench failed"; tail $out/ubench.log; exit 1; }
python $R/util/tuner/tuner.py -s $R/gpurun_out/ubench -b MI355X -o $R/configs/tuned > $out/tuner.log 2>&1 \
  || { echo "tuner failed"; tail $out/tuner.log; exit 1; }
cp -r $R/configs/tuned/AMD_Instinct_MI355X $out/tuned
bash $R/tools/gpu_trace_and_time.sh || exit 1
SUITE=${SUITE:-rodinia_2.0-ft-hip}
export SUITE
if [ "${ENG:-GPU}" = GPU ]; then CFG=MI355X_TUNED-GPU; SLOTS="-g 1 -c 8"; else CFG=MI355X_TUNED; SLOTS="-c 10 --threads 2"; fi
# one GPU-engine simulation per GPU at a time: an MI355X-config simulation
# occupies all 256 CUs (the engine also serialises launches across processes)
export PROCMAN_STATE=$out/procman.json ASIM_JOB_LOGDIR=$out/logs PROCMAN_PER_GPU=1
JL=$R/util/job_launching
timeout -k 10 300 python $JL/run_simulations.py -B $SUITE -C $CFG -T $out/traces -N corr -l local \
  -r $out/simrun $SLOTS > $out/launch.log 2>&1 || { echo "launch failed"; tail $out/launch.log; exit 1; }
timeout -k 10 700 python $JL/monitor_func_test.py -N corr -r $out/simrun -S 10 -T 650 -K -j procman \
  > $out/monitor.log 2>&1; mrc=$?
tail -25 $out/monitor.log
python $JL/get_stats.py -N corr -r $out/simrun -k -K -I > $out/stats_per_kernel.csv
python $JL/get_stats.py -N corr -r $out/simrun -I > $out/stats.csv
python $R/util/plotting/plot-correlation.py -c $out/stats_per_kernel.csv -H $out/hw -B 1 --clock_mhz 2400 \
  -p mi355x -o $out/correl | tee $out/correl.log
# keep the simulator outputs, drop the trace links / copies
find $out/simrun -name traces -type l -delete
# keep each app's traces when its archive is small (local re-simulation)
mkdir -p $out/trace_tgz
for d in $out/traces/*/; do
  a=$(basename $d)
  tar czf $out/trace_tgz/$a.tgz -C $out/traces $a
  sz=$(du -m $out/trace_tgz/$a.tgz | cut -f1)
  [ "$sz" -gt 12 ] && rm -f $out/trace_tgz/$a.tgz && echo "$a traces archive too big ($sz MB), dropped"
done
rm -rf $out/traces
du -sh $out
exit $mrc
