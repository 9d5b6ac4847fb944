#!/bin/bash
# Round-3 final correlation record on the GPU engine with the final tree's
# MI355X model (fetch blocks, LDS lane groups, 64 B L1 lookups).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r3g
timeout -k 10 1000 bash tools/gpu_correlate.sh > gpurun_out/r3g/correlate.log 2>&1
grep -v "^wrote" gpurun_out/corr/correl.log | head -40
