#!/bin/bash
# Round 5: lane-parallel issue A/B (base vs par) + GPU == CPU engine tier on the new build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=abso/base.so B=abso/par.so TAG=par REPS=2 APPS="bfs streamcluster hotspot heartwall backprop" bash tools/gpu_ab_pair.sh || exit $?
mkdir -p gpurun_out/r5ab/par
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_engine.py tests/test_concurrent.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5ab/par/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r5ab/par/pytest.log
exit $rc
