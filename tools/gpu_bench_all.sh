#!/bin/bash
# GPU-box: GPU tests, then the bench with each engine choice (node default,
# GPU engine only, CPU engine job-parallel on the box's cores).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_node.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --engine gpu > gpurun_out/bench_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --engine cpu > gpurun_out/bench_cpu.log 2>&1
tail -1 gpurun_out/bench_node.log
