#!/bin/bash
# Run the CDNA4 micro-benchmark suite (bin/ubench/*) on the current GPU and
# keep each program's output under $1 (default gpurun_out/ubench); every
# program runs under its own time limit and the script stops at the first
# failure (GPU-box etiquette: no retries after a fault).
set -o pipefail
out=${1:-gpurun_out/ubench}
mkdir -p "$out"
for p in ${UBENCH_PROGS:-ub_config ub_cache_lat ub_cache_policy ub_cache_geom ub_l1_assoc ub_alu ub_lds ub_mfma ub_mfma_shapes ub_bw_widths ub_icache ub_atomic_kernel ub_launch ub_mem_bw ub_l2_release ub_kernel_lat_tb ub_l1_adaptive ub_shared_bw ub_atomic_bw ub_dram_atom ub_mem_lat ub_copy_engine ub_regfile ub_power}; do
  echo "== $p"
  timeout -k 10 240 ./bin/ubench/$p > "$out/$p.log" 2>&1 || { echo "$p failed rc=$?"; tail -5 "$out/$p.log"; exit 1; }
  tail -3 "$out/$p.log"
done
echo "== launch latency (rocprofv3 durations of empty kernels)"
timeout -k 10 240 python accel_sim_framework_distributed_amd/hw_stats/launch_latency.py -o "$out/launch_rocprof" \
  > "$out/ub_launch_rocprof.log" 2>&1 || { echo "launch_latency failed"; tail -5 "$out/ub_launch_rocprof.log"; exit 1; }
tail -4 "$out/ub_launch_rocprof.log"
echo "== instruction cache across launches (rocprofv3 SQC counters)"
( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d "$out/icache_launch" \
  -o run -- "$OLDPWD/bin/ubench/ub_icache_launch" > "$out/icache_launch.run.log" 2>&1 ) \
  || { echo "icache launch run failed"; tail -5 "$out/icache_launch.run.log"; exit 1; }
python accel_sim_framework_distributed_amd/hw_stats/icache_launch.py "$out/icache_launch" > "$out/ub_icache_launch.log" \
  || { echo "icache launch parse failed"; exit 1; }
tail -3 "$out/ub_icache_launch.log"
