#!/bin/bash
# Round 5: where the GPU engine's time goes on short-kernel apps: wall time per
# simulated kernel, then the same under rocprofv3 kernel stats (device time of
# engine_kernel vs host time).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/overhead
mkdir -p $out
timeout -k 10 200 python3 $R/tools/engine_overhead.py streamcluster,nw,bfs gpu > $out/wall.txt 2>&1 || { cat $out/wall.txt; exit 1; }
cat $out/wall.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run \
  -- python3 $R/tools/engine_overhead.py streamcluster gpu > $out/prof.log 2>&1 || { tail $out/prof.log; exit 1; }
tail -3 $out/prof.log
cat $(find $out/prof -name "*kernel_stats.csv" | head -1) | cut -c1-220 | head -12
