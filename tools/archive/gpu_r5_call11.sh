#!/bin/bash
# Caching device allocator (no device-synchronising frees between concurrent
# simulations): GPU engine test tier, then the node bench twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5c11
mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $o/node$i.out 2> $o/node$i.err || { tail -5 $o/node$i.err; exit 1; }
  tail -1 $o/node$i.out | cut -c1-200
done
