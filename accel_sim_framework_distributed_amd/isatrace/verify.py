#!/usr/bin/env python3
"""Check automatic ISA traces against the hardware's own instruction counters.

For every traced kernel, the wave-level instruction counts by class in
``kernel-N.traceg`` are compared with rocprofv3 ``SQ_INSTS_*`` / ``SQ_WAVES``
of the *uninstrumented* build of the same source (kernels matched by launch
order).  The classes follow the SQ counter definitions: VALU (``v_*``),
SALU (scalar ALU, without memory / branch / wait / nop / barrier / end),
SMEM (``s_load`` / ``s_buffer_load`` / ``s_dcache``), VMEM_RD / VMEM_WR
(global / buffer / flat / scratch loads (+ atomics) / stores), LDS (``ds_*``)
and BRANCH (``s_branch`` / ``s_cbranch_*``).

    verify.py <trace_dir> <rocprof_pmc_dir>     (prints one row per kernel)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import Counter, defaultdict
from typing import Dict, List

CLASSES = ("WAVES", "VALU", "SALU", "SMEM", "VMEM_RD", "VMEM_WR", "LDS", "BRANCH")
_NOT_SALU = ("s_waitcnt", "s_nop", "s_barrier", "s_endpgm", "s_sleep", "s_setprio", "s_sched", "s_sendmsg",
             "s_trap", "s_icache", "s_ttrace")


def classify(m: str) -> str:
    if m.startswith("v_"):
        return "VALU"
    if m.startswith("ds_"):
        return "LDS"
    if m.startswith(("global_", "buffer_", "flat_", "scratch_")):
        if "store" in m:
            return "VMEM_WR"
        return "VMEM_RD"
    if m.startswith(("s_load", "s_buffer_load", "s_dcache", "s_store", "s_buffer_store", "s_memtime",
                     "s_memrealtime")):
        return "SMEM"
    if m.startswith(("s_branch", "s_cbranch")):
        return "BRANCH"
    if m.startswith(_NOT_SALU):
        return "OTHER"
    if m.startswith("s_"):
        return "SALU"
    return "OTHER"


def trace_counts(path: str) -> Counter:
    c: Counter = Counter()
    with open(path) as f:
        for ln in f:
            if ln.startswith("warp ="):
                c["WAVES"] += 1
                continue
            if not ln or ln[0] in "-#\n" or ln.startswith(("thread block", "insts =")):
                continue
            toks = ln.split()
            if len(toks) < 4:
                continue
            nd = int(toks[2])
            c[classify(toks[3 + nd])] += 1
    return c


def traced_kernels(trace_dir: str) -> List[Counter]:
    kl = os.path.join(trace_dir, "kernelslist.g")
    out = []
    for ln in open(kl):
        s = ln.strip()
        if s.startswith("kernel-") and s.endswith(".traceg"):
            out.append(trace_counts(os.path.join(trace_dir, s)))
    return out


def pmc_kernels(pmc_dir: str) -> List[Dict[str, float]]:
    per: Dict[int, Dict[str, float]] = defaultdict(dict)
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "__amd_rocclr_" in row.get("Kernel_Name", ""):
                continue
            d = int(row["Dispatch_Id"])
            k = row["Counter_Name"].replace("SQ_INSTS_", "").replace("SQ_", "")
            per[d][k] = per[d].get(k, 0.0) + float(row["Counter_Value"])
    return [per[d] for d in sorted(per)]


def compare(trace_dir: str, pmc_dir: str) -> Dict:
    tk, hk = traced_kernels(trace_dir), pmc_kernels(pmc_dir)
    rows = []
    tot_t: Counter = Counter()
    tot_h: Counter = Counter()
    for i in range(min(len(tk), len(hk))):
        r = {"kernel": i + 1}
        for c in CLASSES:
            t, h = tk[i].get(c, 0), hk[i].get(c, float("nan"))
            r[c] = (t, h)
            tot_t[c] += t
            if h == h:
                tot_h[c] += h
        rows.append(r)
    summary = {c: {"trace": tot_t[c], "hw": tot_h[c],
                   "err_pct": (100.0 * (tot_t[c] - tot_h[c]) / tot_h[c]) if tot_h[c] else None} for c in CLASSES}
    return {"kernels": len(rows), "traced": len(tk), "profiled": len(hk), "rows": rows, "total": summary}


def main(argv=None) -> int:
    a = sys.argv[1:] if argv is None else argv
    res = compare(a[0], a[1])
    print(json.dumps(res["total"], indent=1))
    print(f"kernels compared: {res['kernels']} (traced {res['traced']}, profiled {res['profiled']})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
