#!/bin/bash
# Engine iteration on the GPU box: GPU==CPU tests, per-app GPU-engine timings,
# bfs stage profile.  Each step has its own limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${ITER:-iter}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu_engine.log 2>&1
timeout -k 10 300 python tools/app_times.py --engine gpu --config GV100 --out $OUT/apps_gpu.json > $OUT/apps_gpu.log 2>&1
timeout -k 10 200 python tools/profile_engine.py --app ${APP:-bfs} > $OUT/stage.log 2>&1
tail -n 3 $OUT/pytest_gpu_engine.log; grep -v amdgpu.ids $OUT/apps_gpu.log; head -4 $OUT/stage.log
