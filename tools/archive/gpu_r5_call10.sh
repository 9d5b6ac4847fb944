#!/bin/bash
# Power-suite kernel durations at the traced sizes (HW side of the simulated
# cycles behind the power model's activity rates), then the node bench with
# the GIL released during simulator construction.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5c10
mkdir -p $o
timeout -k 10 300 bin/apps/power_suite time > $o/power_suite_time.csv 2> $o/power_suite_time.err || { tail $o/power_suite_time.err; exit 1; }
head -5 $o/power_suite_time.csv
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $o/node.out 2> $o/node.err || { tail -5 $o/node.err; exit 1; }
tail -1 $o/node.out | cut -c1-300
