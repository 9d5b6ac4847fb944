#!/bin/bash
# Round 4, second session, GPU call 2: node bench + GPU-engine-only bench +
# rocprofv3 kernel stats of the bench, then the power suite with the
# cache-resident kernels traced at steady state.  Each step has its own limit;
# the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > $O/bench_node.log 2>&1
tail -1 $O/bench_node.log
timeout -k 10 400 python3 -u bench.py --engine gpu --steps 5 --warmup 2 > $O/bench_gpu.log 2>&1
tail -1 $O/bench_gpu.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --engine gpu --steps 3 --warmup 1 > $O/bench_prof.log 2>&1
find $O/prof -name "*stats*" | head
bash tools/gpu_power_r4c.sh
