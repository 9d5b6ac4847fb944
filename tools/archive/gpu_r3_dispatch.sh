#!/bin/bash
# Streaming ISA capture through the host ring, GPU==CPU bit-exactness of the XCD round-robin dispatch / 64 B store path,
# then the full correlation pipeline on the GPU engine.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3d
mkdir -p $out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_isatrace.py -m gpu -x -v --timeout 240 --timeout-method thread \
  > $out/isat_ring.log 2>&1 || { tail -40 $out/isat_ring.log; exit 1; }
tail -3 $out/isat_ring.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_cdna_memory.py -m gpu -x -v --timeout 240 \
  --timeout-method thread > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -3 $out/gputest.log
bash tools/gpu_correlate.sh
# the round-3 micro-benchmarks (each under its own limit)
cd $R
UBENCH_PROGS="ub_kernel_lat_tb ub_l1_adaptive ub_shared_bw ub_atomic_bw ub_dram_atom ub_mem_lat ub_copy_engine ub_regfile" \
  bash tools/run_ubench.sh gpurun_out/ubench_r3new
