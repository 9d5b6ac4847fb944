#!/bin/bash
# Round 5: the RCCL device kernels a one-GPU communicator runs (every
# collective once and a send / receive pair to itself), rocprofv3 kernel trace.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/rccl_self
mkdir -p $out
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
  -- $R/bin/examples/rccl-self > $out/run.log 2>&1; e=$?
tail -3 $out/run.log
[ $e -eq 0 ] || exit $e
python3 - "$out" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Kernel_Name"][:120], r.get("Grid_Size", ""), r.get("Workgroup_Size", ""), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
PY
