#!/bin/bash
# GPU batch: per-app phase times on both engines (CPU with 1/2/4 threads),
# then the 1-GPU node bench with thread widening.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4b2
timeout -k 10 400 python3 -u tools/app_phases.py --apps hotspot,backprop,heartwall,bfs,srad_v2,streamcluster,nw,lud,pathfinder,nn \
  --engines gpu,cpu --threads 1,2,4 --reps 2 --out gpurun_out/r4b2/app_phases.json > gpurun_out/r4b2/app_phases.log 2>&1
rc=$?; echo "phases rc=$rc"; tail -3 gpurun_out/r4b2/app_phases.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r4b2/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r4b2/bench.log; exit $rc
