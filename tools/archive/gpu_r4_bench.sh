#!/bin/bash
# GPU: the 1-GPU node bench (per-app step wall times in the JSON).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4bench
timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r4bench/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r4bench/bench.log; exit $rc
