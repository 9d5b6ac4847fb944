#!/bin/bash
# Round 5 engine A/B: GPU-engine sim seconds per app (stage profiler off),
# then the GPU == CPU bit-exactness tier of the engine.
# usage: TAG=name [APPS="bfs ..."] [TESTS=1] bash tools/archive/gpu_r5_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5ab/${TAG:-run}
mkdir -p $out
export ASIM_GPU_PROFILE=0
for app in ${APPS:-bfs streamcluster hotspot heartwall backprop nw}; do
  timeout -k 10 120 python3 tools/profile_engine.py --app $app >> $out/times.log 2>&1 || exit $?
done
grep -v amdgpu.ids $out/times.log
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread \
    > $out/pytest.log 2>&1
  rc=$?
  tail -3 $out/pytest.log
  exit $rc
fi
