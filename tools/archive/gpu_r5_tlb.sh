#!/bin/bash
# Round 5: address-translation micro-benchmark (bin/ubench/ub_tlb): same /
# next-kernel / cold pointer-chase latency vs the number of pages a fixed
# number of lines spans.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/ubench
mkdir -p $out
cd /tmp && timeout -k 10 240 $R/bin/ubench/ub_tlb > $out/ub_tlb.log 2>&1; e=$?
cat $out/ub_tlb.log | grep -v "^#"
exit $e
