#!/bin/bash
# GPU-box probe: GPU tests, 1-GPU bench (GPU engine, and the CPU engine
# job-parallel on the box's cores), engine stage profiles of the long apps.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
if [ -n "$CPU_BENCH" ]; then
ASIM_CPU_JOBS=16 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --engine cpu > gpurun_out/bench_cpu16.log 2>&1
fi
for app in ${PROBE_APPS:-streamcluster bfs hotspot}; do
  timeout -k 10 120 python tools/profile_engine.py --app $app > gpurun_out/prof_$app.log 2>&1
done
cat gpurun_out/bench1.log
