#!/bin/bash
# Round 5 benches on one MI355X: the headline (node placement), GPU-engine
# only and CPU-engine only suite runs, then the tuner config sweep
# (BASELINE config #5) on each engine choice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5bench
mkdir -p $o
run() { local name=$1; shift; timeout -k 10 ${T:-300} python3 bench.py "$@" > $o/$name.out 2> $o/$name.err || { echo "$name failed"; tail -5 $o/$name.err; exit 1; }; tail -1 $o/$name.out | cut -c1-400; }
run node --steps 10 --warmup 3
run gpu --engine gpu --steps 3 --warmup 1
run cpu --engine cpu --steps 3 --warmup 1
T=600 run sweep_node --sweep --engine node --steps 1 --warmup 0
T=600 run sweep_cpu --sweep --engine cpu --steps 1 --warmup 0
T=900 run sweep_gpu --sweep --engine gpu --steps 1 --warmup 0
