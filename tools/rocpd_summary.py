#!/usr/bin/env python3
"""Summarise a rocprofv3 (ROCm 7.x) rocpd SQLite database: per-kernel totals
(the `top_kernels` view) as CSV, plus the dispatch geometry of the hottest
kernel.  Used to turn gpurun_out/<run>/*.db into a committed profiles/ file.

    python tools/rocpd_summary.py gpurun_out/prof_bench/run_results.db > profiles/x.csv
"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    w = csv.writer(sys.stdout)
    w.writerow(["name", "calls", "total_us", "avg_us", "percent"])
    for name, calls, tot, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(tot, 3), round(avg, 3), round(pct, 3)])
    r = c.execute("select name, grid_x, workgroup_x, lds_size, vgpr_count, accum_vgpr_count, sgpr_count, "
                  "scratch_size from kernels order by duration desc limit 1").fetchone()
    if r:
        sys.stdout.write("# hottest dispatch: name=%s grid=%s wg=%s lds=%s vgpr=%s agpr=%s sgpr=%s scratch=%s\n" % r)


if __name__ == "__main__":
    main()
