#!/bin/bash
# Round-3 GPU check on the MI355X box: the whole GPU test tier (one process),
# smoke(), the 1-GPU bench, engine-only benches (GPU engine / CPU engine on
# the same box) and a rocprofv3 kernel-stats profile of a short bench run.
# Each step has its own time limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3f
mkdir -p $out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 400 python bench.py > $out/bench_node.log 2>&1
tail -1 $out/bench_node.log
timeout -k 10 400 python bench.py --engine gpu > $out/bench_gpu.log 2>&1
tail -1 $out/bench_gpu.log
timeout -k 10 400 python bench.py --engine cpu > $out/bench_cpu.log 2>&1
tail -1 $out/bench_cpu.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 \
  > $out/prof.log 2>&1
find $out/prof -name "*kernel_stats.csv" | head -3
