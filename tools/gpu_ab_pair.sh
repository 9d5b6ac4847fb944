#!/bin/bash
# In-call engine A/B: the same apps on two builds of _asim, alternating
# A B A B in one process lifetime each, on one box (box-to-box variance of the
# engine's time is up to 1.6x, so A/B across calls is not comparable).
# usage: A=path/to/base.so B=path/to/new.so TAG=name [APPS=...] [REPS=2] bash tools/gpu_ab_pair.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ab/${TAG:-run}
mkdir -p $out
export ASIM_GPU_PROFILE=0
for rep in $(seq 1 ${REPS:-2}); do
  for side in A B; do
    so=${!side}
    for app in ${APPS:-bfs streamcluster hotspot heartwall backprop nw}; do
      echo -n "$side rep$rep " >> $out/times.log
      ASIM_NATIVE_SO=$so timeout -k 10 120 python3 tools/profile_engine.py --app $app 2>&1 | grep -v amdgpu.ids >> $out/times.log || exit $?
    done
  done
done
cat $out/times.log
