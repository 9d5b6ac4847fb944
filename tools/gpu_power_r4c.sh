#!/bin/bash
# Round 4c: power suite with the cache-resident kernels traced at steady state
# (16 L1 passes / 6 L2 passes instead of 2): measure, trace, simulate, fit on
# the single-unit kernels, validate on the held-out mixes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PWR_OUT=power_r4c PWR_HELDOUT=1 PWR_SIM_SECS=700 timeout -k 10 1000 bash tools/gpu_power.sh
