#!/usr/bin/env python3
"""Where the MI355X L2's read requests come from, per app, from a correlation
run's rocprofv3 counters (tools/gpu_correlate.sh hw/ directory): the vector
L1's misses (TCP_TCC_READ_REQ) and the rest of TCC_READ (the SQC's scalar-data
and instruction misses, the command processor's dispatch / kernarg reads),
and how TCC_HIT / TCC_MISS split once the reads that left for the fabric
(TCC_EA0_RDREQ) are known: the gap analysis behind the 'L2 hits' row of the
correlator (profiles/correlation/README.md).

    python tools/l2_read_sources.py [gpurun_out/corr/hw]
"""
import collections
import csv
import glob
import os
import sys


def sums(hw: str, app: str):
    s = collections.defaultdict(float)
    for f in glob.glob(os.path.join(hw, app, "*", "ctr*_0", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            s[r["Counter_Name"]] += float(r["Counter_Value"])
    launches = 0
    for f in glob.glob(os.path.join(hw, app, "*", "run_0", "run_kernel_trace.csv")):
        launches += sum(1 for _ in csv.DictReader(open(f)))
    return s, launches


def main():
    hw = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "gpurun_out", "corr", "hw")
    print(f"{'app':14s} {'launch':>6s} {'TCC_READ':>9s} {'TCP_RD':>8s} {'non-TCP':>8s} {'SMEM':>7s} {'rd_miss':>8s} "
          f"{'rd_hit':>7s} {'WRITE':>7s} {'wr_hit':>7s} {'TCP hit%':>8s}")
    for app in sorted(os.listdir(hw)):
        s, n = sums(hw, app)
        if not s:
            continue
        rd, tcp = s["TCC_READ"], s["TCP_TCC_READ_REQ"]
        rmiss = s["TCC_EA0_RDREQ"]
        rhit = rd - rmiss
        whit = s["TCC_HIT"] - rhit
        lk_rd = s["TCP_TOTAL_CACHE_ACCESSES"] - s["TCP_TCC_WRITE_REQ"]
        l1hit = 100.0 * (1.0 - tcp / lk_rd) if lk_rd > 0 else float("nan")
        print(f"{app:14s} {n:6d} {rd:9.0f} {tcp:8.0f} {rd - tcp:8.0f} {s['SQ_INSTS_SMEM']:7.0f} {rmiss:8.0f} "
              f"{rhit:7.0f} {s['TCC_WRITE']:7.0f} {whit:7.0f} {l1hit:8.1f}")


if __name__ == "__main__":
    main()
