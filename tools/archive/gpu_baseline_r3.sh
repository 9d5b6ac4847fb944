#!/bin/bash
# Round-3 baseline: per-app engine timings (GPU engine, CPU engine) and the
# bfs stage profile on the current tree.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3base
timeout -k 10 300 python tools/app_times.py --engine gpu --config GV100 --out gpurun_out/r3base/apps_gpu.json > gpurun_out/r3base/apps_gpu.log 2>&1
timeout -k 10 300 python tools/app_times.py --engine cpu --config GV100 --out gpurun_out/r3base/apps_cpu.json > gpurun_out/r3base/apps_cpu.log 2>&1
timeout -k 10 200 python tools/profile_engine.py --app bfs > gpurun_out/r3base/stage_bfs.log 2>&1
timeout -k 10 200 python bench.py --engine gpu --steps 3 --warmup 1 > gpurun_out/r3base/bench_gpu.log 2>&1
timeout -k 10 200 python bench.py --engine cpu --steps 3 --warmup 1 > gpurun_out/r3base/bench_cpu.log 2>&1
tail -n 3 gpurun_out/r3base/*.log
