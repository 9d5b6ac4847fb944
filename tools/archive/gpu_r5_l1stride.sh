#!/bin/bash
# Round 5: vector-L1 data path under strided lane addresses (bin/ubench/ub_l1_stride).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/ubench
mkdir -p $out
cd /tmp && timeout -k 10 120 $R/bin/ubench/ub_l1_stride > $out/ub_l1_stride.log 2>&1; e=$?
cat $out/ub_l1_stride.log | grep -v "^#"
exit $e
