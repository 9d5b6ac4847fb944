#!/usr/bin/env python3
"""Merge get_stats CSV files of several simulator builds / launches into one
(reference util/plotting/merge-stats.py:19-148).

Each input is get_stats' block format (one block per stat: ``APPS,<cfg>...``
then ``<app>/<args>--<kernel>,<v>...``).  Configurations are suffixed with the
build they were produced by when the file records one (the ``Accel-Sim-build``
stat, as the reference tags ``<cfg>-accel-<hash>``), a configuration that
appears in more than one file is kept from the first file only (the reference
warns and filters it the same way), and only the stats and app/kernel rows
common to every file are written.  Output goes to stdout, configs as columns
unless ``-R``.

    util/plotting/merge-stats.py -c a.csv,b.csv [-R] > merged.csv
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from typing import Dict, List, Tuple

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching.get_stats import (StatTable, parse_csv_blocks,  # noqa
                                                                            render_csv)
else:
    from ..job_launching.get_stats import StatTable, parse_csv_blocks, render_csv

BUILD_STAT = "Accel-Sim-build"
HASH_RE = re.compile(r"([0-9a-f]{7,40})")


def _build_tag(blocks: Dict[str, Dict[str, Dict[str, str]]]) -> Dict[str, str]:
    """config -> short build hash recorded in the file (if any)."""
    tags: Dict[str, str] = {}
    for stat, rows in blocks.items():
        if not stat.startswith(BUILD_STAT):
            continue
        for row in rows.values():
            for cfg, v in row.items():
                m = HASH_RE.search(v or "")
                if m and v != "NA":
                    tags.setdefault(cfg, m.group(1)[:7])
    return tags


def merge(texts: List[Tuple[str, str]], warn=sys.stderr) -> StatTable:
    """texts: [(name, csv text)] -> merged table."""
    parsed = [(name, parse_csv_blocks(t)) for name, t in texts]
    common_stats = None
    common_rows = None
    for _, blocks in parsed:
        st = [s for s in blocks if not s.startswith(BUILD_STAT)]
        rows = {r for b in blocks.values() for r in b}
        common_stats = st if common_stats is None else [s for s in common_stats if s in st]
        common_rows = rows if common_rows is None else common_rows & rows
    out = StatTable()
    out.stats = list(common_stats or [])
    seen = set()
    for name, blocks in parsed:
        tags = _build_tag(blocks)
        cfgs = []
        for rows in blocks.values():
            for row in rows.values():
                for c in row:
                    if c not in cfgs:
                        cfgs.append(c)
        for c in cfgs:
            full = f"{c}-accel-{tags[c]}" if c in tags else c
            if full in seen:
                print(f"Found redundant config: {full} in csvf: \"{name}\" - filtering it out.", file=warn)
                continue
            seen.add(full)
            for stat in out.stats:
                for rowname, row in blocks.get(stat, {}).items():
                    if rowname not in common_rows or c not in row:
                        continue
                    appargs, _, kernel = rowname.partition("--")
                    out.set(appargs, kernel, full, stat, row[c])
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-c", "--csv_files", required=True, help="comma-separated get_stats CSV files to merge")
    ap.add_argument("-R", "--configs_as_rows", action="store_true")
    a = ap.parse_args(argv)
    texts = []
    for f in a.csv_files.split(","):
        if not f:
            continue
        if not os.path.exists(f):
            print(f"Warning path {f} does not exist. Continuing", file=sys.stderr)
            continue
        print(f"Processing {f}", file=sys.stderr)
        texts.append((f, open(f).read()))
    if not texts:
        return 1
    sys.stdout.write(render_csv(merge(texts), configs_as_rows=a.configs_as_rows))
    return 0


if __name__ == "__main__":
    sys.exit(main())
