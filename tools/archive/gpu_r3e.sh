#!/bin/bash
# Round-3 (session 2) final-tree check: the whole GPU tier, smoke, the 1-GPU
# bench and a rocprofv3 kernel-stats run of a short bench.  Each step has its
# own time limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3e
mkdir -p $out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_node.log 2>&1
tail -1 $out/bench_node.log | cut -c1-300
timeout -k 10 400 python bench.py --engine gpu > $out/bench_gpu.log 2>&1
tail -1 $out/bench_gpu.log | cut -c1-300
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 \
  > $out/prof.log 2>&1
ls $out/prof
