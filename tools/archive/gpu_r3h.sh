#!/bin/bash
# rocprofv3 PMC pass over the matrix-core ingest (tools/ingest_bench.py):
# per-dispatch MFMA / VALU / LDS / SALU instruction counts of ingest_kernel.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3h
mkdir -p $out
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD \
  --output-format csv -d $out/pmc -o run -- python3 $R/tools/ingest_bench.py --reps 1 > $out/pmc.log 2>&1
find $out/pmc -name "*.csv" | head
