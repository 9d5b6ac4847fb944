#!/bin/bash
# GPU: where the L2's non-vector reads come from -- the SQC's (scalar data +
# instruction cache, shared by a CU pair) requests to the L2 next to the
# TCC / TCP read counters, one rocprofv3 pass each, on the correlation suite;
# then the 1-GPU node bench (tools/archive/gpu_r4_bench.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sqc
rm -rf $out && mkdir -p $out
timeout -k 10 500 python3 accel_sim_framework_distributed_amd/hw_stats/run_hw.py -B rodinia_2.0-ft-hip -R 1 \
  -c SQC_TC_INST_REQ,SQC_TC_DATA_READ_REQ,SQC_TC_REQ,SQC_DCACHE_REQ,SQC_DCACHE_HITS,SQC_DCACHE_MISSES,SQC_ICACHE_REQ,SQC_ICACHE_MISSES \
  -c TCC_READ,TCC_REQ,TCC_HIT,TCP_TCC_READ_REQ -o $out/hw > $out/hw.log 2>&1 \
  || { echo "sqc counters failed"; tail -20 $out/hw.log; exit 1; }
echo "sqc counters done"
bash tools/archive/gpu_r4_bench.sh
