#!/bin/bash
# Round 5 final tree: rocprofv3 kernel statistics of one bench.py run.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/final_prof
mkdir -p $out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
  -- python3 $R/bench.py --steps 2 --warmup 1 > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
grep '^{"metric"' $out/bench.log | cut -c1-200
cat $(find $out -name "*kernel_stats.csv" | head -1) | cut -c1-200 | head -12
