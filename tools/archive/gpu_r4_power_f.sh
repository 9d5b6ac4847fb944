#!/bin/bash
# Round 4: power suite (steady-state traces) with the fitted L1 / LDS data paths.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PWR_OUT=power_r4f PWR_HELDOUT=1 PWR_SIM_SECS=600 timeout -k 10 900 bash tools/gpu_power.sh
