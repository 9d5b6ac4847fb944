#!/bin/bash
# Round 4, call 4: GPU tests, smoke, node bench (10 steps), then the power
# suite re-simulated with the vector-L1 data path (steady-state traces).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 3 > $O/bench_node.log 2>&1
tail -1 $O/bench_node.log
PWR_OUT=power_r4e PWR_HELDOUT=1 PWR_SIM_SECS=500 timeout -k 10 700 bash tools/gpu_power.sh > $O/power.log 2>&1
tail -3 $O/power.log
