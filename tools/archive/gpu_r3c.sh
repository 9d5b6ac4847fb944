#!/bin/bash
# Round-3 (session 2) GPU step: the matrix-core ingest tests and bench, the
# whole GPU tier, smoke, the 1-GPU bench, a rocprofv3 kernel-stats run of the
# ingest, then the micro-benchmarks added this round.  Each step has its own
# time limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3c
mkdir -p $out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ingest_mfma.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_ingest.log 2>&1
tail -2 $out/pytest_ingest.log
timeout -k 10 300 python -u tools/ingest_bench.py --big --out $out/ingest_bench_big.json > $out/ingest_bench_big.log 2>&1
python -c "import json; print(json.load(open('$out/ingest_bench_big.json'))['total'])"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench_node.log 2>&1
tail -1 $out/bench_node.log | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_ingest -o run -- python3 $R/tools/ingest_bench.py --big --reps 1 \
  > $out/prof_ingest.log 2>&1
find $out/prof_ingest -name "*kernel_stats.csv" | head -3
cd $R
UBENCH_PROGS="ub_kernel_lat_tb ub_l1_adaptive ub_shared_bw ub_atomic_bw ub_dram_atom ub_mem_lat ub_copy_engine ub_regfile" \
  bash tools/run_ubench.sh $out/ubench > $out/ubench_run.log 2>&1
tail -20 $out/ubench_run.log
