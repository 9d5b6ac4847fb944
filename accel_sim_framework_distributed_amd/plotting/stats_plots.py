#!/usr/bin/env python3
"""Plot / merge get_stats CSVs (reference util/plotting/plot-get-stats.py:65-79
and merge-stats.py:101-104).

    stats_plots.py plot  -c stats.csv [-o out_dir]        # one bar chart per stat
    stats_plots.py merge -c a.csv -c b.csv [-o merged.csv] # union of configs / rows
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import OrderedDict
from typing import Dict, List

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import get_stats  # noqa: E402
    from accel_sim_framework_distributed_amd.plotting import svg  # noqa: E402
else:
    from ..job_launching import get_stats
    from . import svg


def merge(csvs: List[str]) -> str:
    """Union of the stat blocks of several CSVs; later files win on clashes."""
    merged: "OrderedDict[str, OrderedDict[str, OrderedDict[str, str]]]" = OrderedDict()
    cfgs: "OrderedDict[str, None]" = OrderedDict()
    for p in csvs:
        for stat, rows in get_stats.parse_csv_blocks(open(p).read()).items():
            blk = merged.setdefault(stat, OrderedDict())
            for row, vals in rows.items():
                blk.setdefault(row, OrderedDict()).update(vals)
                for c in vals:
                    cfgs[c] = None
    cl = list(cfgs)
    out = []
    for stat, rows in merged.items():
        out.append("-" * 100 + "," * len(cl))
        out.append(stat + "," * len(cl))
        out.append(",".join(["APPS"] + cl))
        for row, vals in rows.items():
            out.append(",".join([row] + [vals.get(c, "NA") for c in cl]))
    return "\n".join(out) + "\n"


def plot(csv_path: str, out_dir: str) -> List[str]:
    os.makedirs(out_dir, exist_ok=True)
    files = []
    for i, (stat, rows) in enumerate(get_stats.parse_csv_blocks(open(csv_path).read()).items()):
        groups = list(rows)
        cfgs: List[str] = []
        for v in rows.values():
            for c in v:
                if c not in cfgs:
                    cfgs.append(c)
        series: Dict[str, List] = {}
        numeric = False
        for c in cfgs:
            col = []
            for g in groups:
                try:
                    col.append(float(rows[g].get(c, "")))
                    numeric = True
                except ValueError:
                    col.append(None)
            series[c] = col
        if not numeric:
            continue
        p = os.path.join(out_dir, f"stat{i:03d}.html")
        with open(p, "w") as f:
            f.write(svg.page(stat, [f"<h3>{stat}</h3>", svg.bars(groups, series, stat, "value")]))
        files.append(p)
    return files


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("cmd", choices=["plot", "merge"])
    ap.add_argument("-c", "--csv", action="append", required=True)
    ap.add_argument("-o", "--out", default="")
    o = ap.parse_args(argv)
    if o.cmd == "merge":
        text = merge(o.csv)
        if o.out:
            open(o.out, "w").write(text)
        else:
            sys.stdout.write(text)
    else:
        for f in plot(o.csv[0], o.out or "stats-html"):
            print("wrote", f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
