#!/usr/bin/env python3
"""Collect AccelWattch power reports into per-configuration CSV tables
(reference util/accelwattch/gen_sim_power_csv.py:43-233).

Input layout (as the reference's collect_power_reports.sh leaves it):
``<reports>/<config>/<benchmark>.log``, each log an
``accelwattch_power_report.log`` with one block per kernel launch.  For every
benchmark the per-component average power of all launches of its first
kernel name (``<bench>_k1``) and, when the app has one, of its second kernel
name (``<bench>_k2``) are averaged; DRAM power absorbs the memory controller
and the L2 absorbs the NoC, as in the reference's table (gen_sim_power_csv.py:215-216).
Components the model variant does not use are dropped like the reference
does per config family (SASS: MC/TC/INT_MUL24/INT_MUL32/INT_DIV/FP_DIV/DP_DIV/NOC;
PTX: MC/NOC; HW/HYBRID: IC/RF).  Unlike the reference, kernel names are taken
from the logs (first-seen order), not from a hard-coded table, so any suite
(the MI355X ub_power kernels included) works.

    util/accelwattch/gen_sim_power_csv.py <reports_dir> [config|all] [-o accelwattch_results]
"""
from __future__ import annotations

import argparse
import csv
import os
import sys
from collections import OrderedDict
from typing import Dict, List

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.power.report import COMPONENTS, parse_power_report  # noqa: E402
else:
    from .report import COMPONENTS, parse_power_report

DROP = {
    "sass": {"MCP", "TCP", "INT_MUL24P", "INT_MUL32P", "INT_DIVP", "FP_DIVP", "DP_DIVP", "NOCP"},
    "ptx": {"MCP", "NOCP"},
    "hw": {"ICP", "RFP"},
}


def _family(config: str) -> str:
    c = config.lower()
    if "hw" in c or "hybrid" in c:
        return "hw"
    if "ptx" in c:
        return "ptx"
    return "sass"


def benchmark_rows(log_text: str, bench: str, config: str) -> "OrderedDict[str, Dict[str, float]]":
    kernels = parse_power_report(log_text)
    names: List[str] = []
    for k in kernels:
        if k["kernel_name"] not in names:
            names.append(k["kernel_name"])
    rows: "OrderedDict[str, Dict[str, float]]" = OrderedDict()
    drop = DROP[_family(config)]
    for idx, name in enumerate(names[:2], 1):
        ks = [k for k in kernels if k["kernel_name"] == name]
        row: Dict[str, float] = OrderedDict()
        for comp in COMPONENTS:
            row[comp] = sum(k["avg"].get(comp, 0.0) for k in ks) / len(ks)
        row["kernel_avg_power"] = sum(k.get("kernel_avg_power", 0.0) for k in ks) / len(ks)
        row["DRAMP"] += row["MCP"]
        row["L2CP"] += row["NOCP"]
        for comp in drop:
            row.pop(comp, None)
        rows[f"{bench}_k{idx}"] = row
    return rows


def collect(reports_dir: str, config: str) -> "OrderedDict[str, Dict[str, float]]":
    d = os.path.join(reports_dir, config)
    table: "OrderedDict[str, Dict[str, float]]" = OrderedDict()
    for fn in sorted(os.listdir(d)):
        if not fn.endswith(".log"):
            continue
        bench = fn[:-4]
        rows = benchmark_rows(open(os.path.join(d, fn)).read(), bench, config)
        if not rows:
            print(f"Warning: {bench} has no simulator data.", file=sys.stderr)
        table.update(rows)
    return table


def write_csv(table: "OrderedDict[str, Dict[str, float]]", path: str) -> None:
    cols: List[str] = []
    for row in table.values():
        for k in row:
            if k not in cols:
                cols.append(k)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow([""] + cols)
        for name, row in table.items():
            w.writerow([name] + [f"{row.get(k, 0.0):.6g}" for k in cols])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("reports", help="directory holding <config>/<benchmark>.log power reports")
    ap.add_argument("config", nargs="?", default="all", help="one config directory name, or 'all'")
    ap.add_argument("-o", "--out", default="accelwattch_results")
    a = ap.parse_args(argv)
    configs = sorted(os.listdir(a.reports)) if a.config == "all" else [a.config]
    os.makedirs(a.out, exist_ok=True)
    for cfg in configs:
        if not os.path.isdir(os.path.join(a.reports, cfg)):
            continue
        print(f"Collecting AccelWattch power results for {cfg}")
        write_csv(collect(a.reports, cfg), os.path.join(a.out, f"accelwattch_{cfg}.csv"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
