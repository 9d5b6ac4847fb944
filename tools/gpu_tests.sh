#!/bin/bash
# GPU test tier (one process), then smoke; each step under its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${ITER:-tests}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -n 5 $OUT/pytest_gpu.log; tail -n 2 $OUT/smoke.log
