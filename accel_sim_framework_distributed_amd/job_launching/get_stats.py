#!/usr/bin/env python3
"""Scrape simulator outputs of a launch into CSV (reference util/job_launching/get_stats.py).

The stats are regexes from a stats YAML (``stats/example_stats.yml``:
``collect_aggregate`` values are cumulative and are differenced per kernel,
``collect_abs`` / ``collect_rates`` are taken as printed).  The CSV layout is
the reference's block format -- one block per stat::

    ----...----,,
    <stat regex>,,
    APPS,<cfg1>,<cfg2>
    <app>/<argfolder>--<kernel>,<v1>,<v2>

(``-R`` transposes to configs-as-rows), so the correlator and plotting tools
read both frameworks' files.  Jobs come from a launch log (``-l``/``-N``) or
from ``-B``/``-C`` lists.
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import yaml

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import common, job_status  # noqa: E402
else:
    from . import common, job_status

EXIT_RE = re.compile(r"GPGPU-Sim: \*\*\* exit detected \*\*\*")
BREAK_RE = re.compile(r"GPGPU-Sim: \*\* break due to reaching the maximum cycles")
KNAME_RE = re.compile(r"kernel_name\s+=\s+(.*)")
BUILD_RE = re.compile(r"^(Accel-Sim\S*\s*\[.*\])")


class StatTable:
    """values[(appargs, kernel)][config][stat] plus the ordering of each axis."""

    def __init__(self):
        self.stats: List[str] = []
        self.configs: List[str] = []
        self.rows: "OrderedDict[str, List[str]]" = OrderedDict()   # appargs -> kernels
        self.values: Dict[Tuple[str, str, str, str], str] = {}

    def add_row(self, appargs: str, kernel: str) -> None:
        ks = self.rows.setdefault(appargs, [])
        if kernel not in ks:
            ks.append(kernel)

    def set(self, appargs, kernel, config, stat, v) -> None:
        self.add_row(appargs, kernel)
        if config not in self.configs:
            self.configs.append(config)
        self.values[(appargs, kernel, config, stat)] = v

    def get(self, appargs, kernel, config, stat, default=None):
        return self.values.get((appargs, kernel, config, stat), default)


def load_stats_yml(path: str) -> Dict[str, List[str]]:
    path = path or os.path.join(common.HERE, "stats", "example_stats.yml")
    y = yaml.safe_load(open(path))
    return {k: list(y.get(k) or []) for k in ("collect_aggregate", "collect_abs", "collect_rates")}


def _compiled(spec):
    out = []
    for kind, key in (("agg", "collect_aggregate"), ("abs", "collect_abs"), ("rate", "collect_rates")):
        for s in spec[key]:
            out.append((s, re.compile(s), kind))
    return out


def parse_output(text: str, spec, per_kernel: bool, kernel_instance: bool) -> Tuple[Dict[str, Dict[str, str]], List[str]]:
    """{kernel: {stat: value}} for one output file, plus kernel order."""
    pats = _compiled(spec)
    res: "OrderedDict[str, Dict[str, str]]" = OrderedDict()
    build = None
    if not per_kernel:
        found = {}
        for line in reversed(text.splitlines()):
            for name, rx, _ in pats:
                if name in found:
                    continue
                m = rx.search(line.rstrip())
                if m:
                    found[name] = m.group(1).strip()
            if build is None:
                mb = BUILD_RE.match(line)
                if mb:
                    build = mb.group(1)
        if build:
            found["Accel-Sim-build"] = build
        res["final_kernel"] = found
        return res, ["final_kernel"]
    cur = None
    counts: Dict[str, int] = {}
    last_raw: Dict[str, float] = {}
    for line in text.splitlines():
        if BREAK_RE.match(line) and cur is not None:
            res.pop(cur, None)   # incomplete kernel
            continue
        mk = KNAME_RE.match(line)
        if mk:
            name = mk.group(1).strip()
            if kernel_instance:
                counts[name] = counts.get(name, -1) + 1
                name += f"--{counts[name]}"
            cur = name
            d = res.setdefault(cur, {})
            d["k-count"] = str(int(d.get("k-count", "0")) + 1)
            continue
        if cur is None:
            continue
        for sname, rx, kind in pats:
            m = rx.search(line.rstrip())
            if not m:
                continue
            v = m.group(1).strip()
            if kind == "agg":
                try:
                    f = float(v)
                except ValueError:
                    res[cur][sname] = v
                    continue
                delta = f - last_raw.get(sname, 0.0)
                last_raw[sname] = f
                prev = float(res[cur].get(sname, 0.0))
                res[cur][sname] = _fmt(prev + delta)
            else:
                res[cur][sname] = v
    return res, list(res.keys())


def _fmt(x: float) -> str:
    return str(int(x)) if float(x).is_integer() else f"{x:.6g}"


def collect(log: Optional[str], run_dir: str, spec, per_kernel: bool = False, kernel_instance: bool = False,
            jobs: Optional[List[Dict]] = None, ignore_failures: bool = False) -> StatTable:
    t = StatTable()
    t.stats = ["Accel-Sim-build"] + [s for k in ("collect_aggregate", "collect_abs", "collect_rates") for s in spec[k]]
    if jobs is None:
        jobs = job_status.parse_log(log)
    for j in jobs:
        d = os.path.join(run_dir, j["app"].replace("/", "_"), j["args"], j["config"])
        outf = _find_output(d, j)
        appargs = f"{j['app']}/{j['args']}"
        if j["config"] not in t.configs:
            t.configs.append(j["config"])
        if outf is None:
            t.add_row(appargs, "final_kernel" if not per_kernel else "NA")
            continue
        text = open(outf, errors="replace").read()
        if not EXIT_RE.search(text):
            print(f"WARNING - {outf} has no exit string; output potentially invalid", file=sys.stderr)
            if not ignore_failures:
                t.add_row(appargs, "final_kernel" if not per_kernel else "NA")
                continue
        kstats, order = parse_output(text, spec, per_kernel, kernel_instance)
        for k in order:
            for s, v in kstats[k].items():
                t.set(appargs, k, j["config"], s, v)
    if per_kernel:
        t.stats.insert(1, "k-count")
    return t


def _find_output(d: str, j: Dict) -> Optional[str]:
    if "jobid" in j:
        p = os.path.join(d, f"{j['name']}.o{j['jobid']}")
        return p if os.path.exists(p) else None
    # -B/-C mode: newest *.o<id> in the directory
    if not os.path.isdir(d):
        return None
    cands = [os.path.join(d, f) for f in os.listdir(d) if re.search(r"\.o\w+$", f)]
    return max(cands, key=os.path.getmtime) if cands else None


def render_csv(t: StatTable, configs_as_rows: bool = False, do_averages: bool = False) -> str:
    out = []
    rows = [(a, k) for a, ks in t.rows.items() for k in ks]
    for stat in t.stats:
        if not any(t.get(a, k, c, stat) is not None for a, k in rows for c in t.configs):
            continue
        ncomma = (len(rows) if configs_as_rows else len(t.configs)) + (1 if do_averages else 0)
        out.append("-" * 100 + "," * ncomma)
        out.append(stat + "," * ncomma)
        if configs_as_rows:
            hdr = ["CFG"] + [f"{a}--{k}" for a, k in rows] + (["AVG"] if do_averages else [])
            out.append(",".join(hdr))
            for c in t.configs:
                vals = [t.get(a, k, c, stat, "NA") for a, k in rows]
                out.append(",".join([c] + vals + ([_avg(vals)] if do_averages else [])))
        else:
            out.append(",".join(["APPS"] + t.configs))
            for a, k in rows:
                out.append(",".join([f"{a}--{k}"] + [t.get(a, k, c, stat, "NA") for c in t.configs]))
            if do_averages:
                out.append(",".join(["AVG"] + [_avg([t.get(a, k, c, stat, "NA") for a, k in rows])
                                                for c in t.configs]))
    return "\n".join(out) + "\n"


def _avg(vals: List[str]) -> str:
    xs = []
    for v in vals:
        try:
            xs.append(float(v))
        except (TypeError, ValueError):
            pass
    return f"{sum(xs) / len(xs):.1f}" if xs else "NA"


def parse_csv_blocks(text: str) -> Dict[str, Dict[str, Dict[str, str]]]:
    """Inverse of render_csv (configs-as-columns): {stat: {row: {config: value}}}."""
    blocks: Dict[str, Dict[str, Dict[str, str]]] = {}
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        if lines[i].startswith("-" * 20):
            stat = lines[i + 1].rstrip(",")
            hdr = lines[i + 2].split(",")
            i += 3
            rows: Dict[str, Dict[str, str]] = {}
            while i < len(lines) and not lines[i].startswith("-" * 20):
                f = lines[i].split(",")
                if f and f[0]:
                    rows[f[0]] = dict(zip(hdr[1:], f[1:]))
                i += 1
            blocks[stat] = rows
        else:
            i += 1
    return blocks


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-l", "--logfile", default="")
    ap.add_argument("-r", "--run_dir", default="")
    ap.add_argument("-N", "--sim_name", default="")
    ap.add_argument("-B", "--benchmark_list", default="")
    ap.add_argument("-C", "--configs_list", default="")
    ap.add_argument("-s", "--stats_yml", default="")
    ap.add_argument("-k", "--per_kernel", action="store_true")
    ap.add_argument("-K", "--kernel_instance", action="store_true")
    ap.add_argument("-R", "--configs_as_rows", action="store_true")
    ap.add_argument("-I", "--ignore_failures", action="store_true")
    ap.add_argument("-A", "--do_averages", action="store_true")
    o = ap.parse_args(argv)
    run_dir = os.path.abspath(o.run_dir) if o.run_dir else os.path.join(common.REPO_ROOT, "sim_run")
    spec = load_stats_yml(o.stats_yml)
    if o.benchmark_list and o.configs_list:
        reg = common.Registry()
        jobs = []
        for _, _, app, args_list in reg.benchmarks(o.benchmark_list.split(",")):
            for a in args_list:
                for c in o.configs_list.split(","):
                    jobs.append(dict(app=app, args=common.argfoldername(a.get("args")), config=c))
        t = collect(None, run_dir, spec, o.per_kernel or o.kernel_instance, o.kernel_instance, jobs=jobs,
                    ignore_failures=o.ignore_failures)
    else:
        log = job_status.logfiles(o.logfile, o.sim_name)[0]
        t = collect(log, run_dir, spec, o.per_kernel or o.kernel_instance, o.kernel_instance,
                    ignore_failures=o.ignore_failures)
    sys.stdout.write(render_csv(t, o.configs_as_rows, o.do_averages))
    return 0


if __name__ == "__main__":
    sys.exit(main())
