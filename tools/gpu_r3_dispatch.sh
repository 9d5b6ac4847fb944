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
