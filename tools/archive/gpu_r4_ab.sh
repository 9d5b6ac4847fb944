#!/bin/bash
# A/B of engine variants on the same box: every app of APPS on the GPU engine
# under each setting of VAR (an environment variable), plain timing (no
# profiler), then the GPU engine's bit-exactness tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ab${TAG:+_$TAG}
mkdir -p $OUT
export ASIM_GPU_PROFILE=0
for rep in 1 2; do
  for val in ${VALS:-lds const}; do
    for app in ${APPS:-bfs hotspot heartwall}; do
      env ${VAR:-ASIM_GPU_CFG}=$val timeout -k 10 150 python3 tools/profile_engine.py --app $app > $OUT/${app}_${val}_$rep.log 2>&1
      grep "KIPS" $OUT/${app}_${val}_$rep.log | sed "s/^/[$val rep$rep] /"
    done
  done
done
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_engine.log 2>&1
  tail -3 $OUT/pytest_gpu_engine.log
fi
