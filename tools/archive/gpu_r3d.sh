#!/bin/bash
# Round-3 (session 2): correlation run of the MI355X config with the CDNA4
# LDS lane-group model (tools/gpu_correlate.sh on the GPU engine), then the
# 1-GPU bench with the ingest size threshold.  Each step has its own time
# limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r3d
timeout -k 10 1000 bash tools/gpu_correlate.sh > gpurun_out/r3d/correlate.log 2>&1
head -3 gpurun_out/corr/correl.log
grep -E "LDS bank|^Cycles" gpurun_out/corr/correl.log
timeout -k 10 400 python bench.py > gpurun_out/r3d/bench_node.log 2>&1
tail -1 gpurun_out/r3d/bench_node.log | cut -c1-300
