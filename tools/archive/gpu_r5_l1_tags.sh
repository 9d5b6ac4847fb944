#!/bin/bash
# Round 5: how the vector L1's TCP_TOTAL_CACHE_ACCESSES counts a wave-load:
# ub_l1_stride (4-byte loads, lanes 4..128 B apart) under a rocprofv3 counter
# pass; per dispatch the counter over the wave-loads it ran.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/l1_tags
mkdir -p $out
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum \
  --output-format csv -d $out -o run -- $R/bin/ubench/ub_l1_stride > $out/run.log 2>&1; e=$?
tail -3 $out/run.log
[ $e -eq 0 ] || exit $e
python3 - "$out" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        per[d]["grid"] = r.get("Grid_Size", "")
for d in sorted(per):
    print(d, {k: v for k, v in per[d].items()})
PY
