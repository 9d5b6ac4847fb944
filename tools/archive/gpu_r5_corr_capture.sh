#!/bin/bash
# Round 5: the GPU half of tools/gpu_correlate.sh -- micro-benchmarks, ISA
# traces of the HIP suite and rocprofv3 timings / counters (4 runs) -- with
# the traces archived for the host half (tuner + simulation + correlator:
# tools/local_full_correlate.sh after util/tuner/tuner.py on the ubench logs).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/corr
rm -rf $out && mkdir -p $out
UBENCH_PROGS="ub_config ub_bw_widths ub_cache_lat ub_cache_policy ub_alu ub_wave_issue ub_lds ub_mfma ub_mfma_shapes ub_icache ub_atomic_kernel ub_launch ub_mem_bw ub_l2_release ub_kernel_lat_tb ub_copy_engine ub_regfile ub_l1_stride ub_mem_lat" \
  bash $R/tools/run_ubench.sh $out/ubench > $out/ubench.log 2>&1 || { echo "ubench failed"; tail $out/ubench.log; exit 1; }
echo "ubench done"
bash $R/tools/gpu_trace_and_time.sh || exit 1
mkdir -p $out/trace_tgz
for d in $out/traces/*/; do
  a=$(basename $d)
  tar czf $out/trace_tgz/$a.tgz -C $out/traces $a
done
rm -rf $out/traces
du -sh $out
