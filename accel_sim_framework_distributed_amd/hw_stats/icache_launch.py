#!/usr/bin/env python3
"""Is the instruction cache cold at every kernel launch?

Reads the rocprofv3 counter run of ``bin/ubench/ub_icache_launch`` (four
back-to-back launches of one ~6 KB kernel, SQC_ICACHE_MISSES per dispatch)
and prints the tuner's option: the dispatch invalidates the SQC when the
later launches miss about as often as the first (within a quarter of it),
``-sim_sqc_invalidate_at_launch 1``; otherwise 0.

    icache_launch.py <rocprofv3 output dir>  > gpurun_out/ubench/ub_icache_launch.log
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict
from typing import Dict, List


def misses_per_dispatch(run_dir: str, kernel: str = "icl_kernel") -> List[float]:
    per: Dict[int, Dict[str, float]] = defaultdict(dict)
    for f in glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            d = int(row["Dispatch_Id"])
            per[d][row["Counter_Name"]] = per[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return [per[d].get("SQC_ICACHE_MISSES", 0.0) for d in sorted(per)]


def verdict(m: List[float]) -> int:
    if len(m) < 2 or m[0] <= 0:
        raise ValueError("need at least two dispatches with misses")
    later = sum(m[1:]) / len(m[1:])
    return 1 if later >= 0.75 * m[0] else 0


def main(argv=None) -> int:
    a = sys.argv[1:] if argv is None else argv
    m = misses_per_dispatch(a[0])
    print("icache misses per launch: " + " ".join(f"{x:.0f}" for x in m))
    v = verdict(m)
    print(f"# icache_misses_first_launch {m[0]:.0f}")
    print(f"# icache_misses_later_launches {sum(m[1:]) / max(1, len(m) - 1):.1f}")
    print(f"-sim_sqc_invalidate_at_launch {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
