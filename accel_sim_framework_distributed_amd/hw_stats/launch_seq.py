#!/usr/bin/env python3
"""Launch-timing model terms from ``bin/ubench/ub_launch_seq`` (run under
``rocprofv3 --kernel-trace --hip-runtime-trace``).

The correlator's hardware cycles are a kernel's rocprofv3 duration (End -
Start timestamp).  For an isolated kernel that is the launch latency plus the
kernel's execution; for a kernel queued right behind another one, or launched
after a copy, it is not obvious what the two timestamps bracket.  The
micro-benchmark stamps every launch's execution window on the device's
100 MHz clock (first wave start, last wave end), so per launch:

  dur      rocprofv3 End - Start
  span     device last-wave end - first-wave start (the work itself)
  over     dur - span: what the duration holds besides the work
  rp_gap   Start - previous kernel's End (rocprofv3 clock; < 0: the start
           stamp precedes the previous kernel's end)
  dev_gap  first-wave start - previous kernel's last-wave end (device clock):
           the dispatch gap between two kernels' execution
  sub_gap  hipLaunchKernel call start - previous call's start (host)
  sub2st   Start - this launch's hipLaunchKernel call start

Per scenario the medians are printed and written as JSON; ``fit()`` turns
them into the simulator's launch options (printed as ``suggest_`` lines the
tuner reads):

  -gpgpu_kernel_launch_latency         idle launch: over of an idle kernel
  -gpgpu_kernel_launch_latency_queued  dev_gap of a kernel queued behind a
                                       running one, plus the end overhead
  -sim_queued_start_overlap 1          when rp_gap < 0 for queued kernels:
                                       the duration of a queued kernel starts
                                       when the previous kernel's last
                                       workgroup was dispatched
  -sim_host_launch_interval            host submission interval of a chain
                                       of launches (sub_gap)

    launch_seq.py -o gpurun_out/ubench/launch_seq          # run + analyse
    launch_seq.py -i gpurun_out/ubench/launch_seq          # analyse a run
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict
from typing import Dict, List

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _rows(run_dir: str, pattern: str) -> List[Dict[str, str]]:
    out: List[Dict[str, str]] = []
    for f in glob.glob(os.path.join(run_dir, "**", pattern), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def load(run_dir: str, log: str) -> List[Dict]:
    """One record per launch of the benchmark, in launch order."""
    tags: Dict[int, tuple] = {}
    stamps: Dict[int, tuple] = {}
    gaps: List[float] = []
    mhz = 0.0
    with open(log) as fh:
        for line in fh:
            p = line.split()
            if not p:
                continue
            if p[0] == "L" and len(p) == 4:
                tags[int(p[1])] = (p[2], float(p[3]))
            elif p[0] == "S" and len(p) == 4:
                stamps[int(p[1])] = (int(p[2]), int(p[3]))
            elif p[0] == "G":
                gaps.append(float(p[1]))
            elif line.startswith("# measured_shader_mhz"):
                mhz = float(p[-1])
    kt = [r for r in _rows(run_dir, "*kernel_trace.csv") if r.get("Kernel_Name", "").lstrip().startswith("ls_")]
    kt.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    kt = kt[1:]  # the clock warm-up launch
    api = {}
    for r in _rows(run_dir, "*hip_api_trace.csv"):
        if "LaunchKernel" in r.get("Function", "") or "ModuleLaunchKernel" in r.get("Function", ""):
            try:
                api[int(r["Correlation_Id"])] = int(r["Start_Timestamp"])
            except (KeyError, ValueError):
                pass
    recs = []
    for i, r in enumerate(kt):
        if i not in tags or i not in stamps:
            continue
        ts, te = stamps[i]
        rec = dict(id=i, scen=tags[i][0], work_us=tags[i][1], start=int(r["Start_Timestamp"]),
                   end=int(r["End_Timestamp"]), ts=ts * 10, te=te * 10)
        cid = r.get("Correlation_Id")
        if cid is not None and cid.isdigit() and int(cid) in api:
            rec["sub"] = api[int(cid)]
        recs.append(rec)
    for j, rec in enumerate(recs):
        rec["dur"] = rec["end"] - rec["start"]
        rec["span"] = rec["te"] - rec["ts"]
        rec["over"] = rec["dur"] - rec["span"]
        if j:
            pr = recs[j - 1]
            rec["rp_gap"] = rec["start"] - pr["end"]
            rec["dev_gap"] = rec["ts"] - pr["te"]
            if "sub" in rec and "sub" in pr:
                rec["sub_gap"] = rec["sub"] - pr["sub"]
        if "sub" in rec:
            rec["sub2st"] = rec["start"] - rec["sub"]
    return recs, mhz, gaps


def summarize(recs: List[Dict]) -> Dict[str, Dict[str, float]]:
    """Medians (ns) per scenario key: scenario/work, pairs split by A's time."""
    groups: Dict[str, List[Dict]] = defaultdict(list)
    prev = None
    chain_pos = 0
    for rec in recs:
        s = rec["scen"]
        if s == "pair_b" and prev is not None:
            key = f"pair_b/A{prev['work_us']:g}/W{rec['work_us']:g}"
        elif s == "chain":
            chain_pos = chain_pos + 1 if prev is not None and prev["scen"] == "chain" and \
                prev["work_us"] == rec["work_us"] and chain_pos < 23 else 0
            key = f"chain/W{rec['work_us']:g}/" + ("first" if chain_pos == 0 else "rest")
        elif s in ("copy_k", "copy_k2", "d2h_k", "gap", "pair_a", "idle"):
            key = f"{s}/W{rec['work_us']:g}"
        else:
            key = s
        groups[key].append(rec)
        prev = rec
    out = {}
    for k, v in groups.items():
        d = {"n": len(v)}
        for f in ("dur", "span", "over", "rp_gap", "dev_gap", "sub_gap", "sub2st"):
            xs = [r[f] for r in v if f in r]
            if xs:
                d[f] = float(np.median(xs))
        out[k] = d
    return out


def gap_series(recs: List[Dict]) -> List[Dict[str, float]]:
    """ls_gap: per host gap (in launch order, 16 launches each) the medians."""
    g = [r for r in recs if r["scen"] == "gap"]
    out = []
    for i in range(0, len(g), 16):
        blk = g[i + 1:i + 16]
        if blk:
            out.append({f: float(np.median([r[f] for r in blk if f in r])) for f in
                        ("dur", "over", "rp_gap", "dev_gap", "sub_gap") if any(f in r for r in blk)})
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-o", "--out", default=os.path.join(REPO, "gpurun_out", "ubench", "launch_seq"))
    ap.add_argument("-i", "--input", default="", help="existing run directory (with ub_launch_seq.log)")
    ap.add_argument("--exe", default=os.path.join(REPO, "bin", "ubench", "ub_launch_seq"))
    ap.add_argument("-j", "--json", default="")
    o = ap.parse_args(argv)
    run_dir = o.input or o.out
    log = os.path.join(run_dir, "ub_launch_seq.log")
    if not o.input:
        os.makedirs(run_dir, exist_ok=True)
        cmd = ["timeout", "-k", "10", "180", "rocprofv3", "--kernel-trace", "--hip-runtime-trace",
               "--output-format", "csv", "-d", run_dir, "-o", "run", "--", o.exe]
        env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
        with open(log, "w") as fh:
            p = subprocess.run(cmd, cwd="/tmp", env=env, stdout=fh, stderr=subprocess.STDOUT, text=True)
        if p.returncode != 0:
            print(open(log).read()[-2000:], file=sys.stderr)
            return p.returncode
    recs, mhz, gaps = load(run_dir, log)
    if not recs:
        print("launch_seq: no ls_* dispatches matched", file=sys.stderr)
        return 1
    mhz = mhz or 2400.0
    summ = summarize(recs)
    cols = ("n", "dur", "span", "over", "rp_gap", "dev_gap", "sub_gap", "sub2st")
    print(f"{'scenario':28s} " + " ".join(f"{c:>9s}" for c in cols) + "   (ns, medians)")
    for k in sorted(summ):
        d = summ[k]
        print(f"{k:28s} " + " ".join(f"{d[c]:9.0f}" if c in d else f"{'-':>9s}" for c in cols))
    gs = gap_series(recs)
    for g, d in zip(gaps, gs):
        print(f"host gap {g:5.1f} us: " + " ".join(f"{k} {v:8.0f}" for k, v in d.items()))
    res = dict(mhz=mhz, scenarios=summ, gap_series=[dict(gap_us=g, **d) for g, d in zip(gaps, gs)])
    if o.json:
        with open(o.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
