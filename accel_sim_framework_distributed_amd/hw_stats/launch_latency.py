#!/usr/bin/env python3
"""Fit the simulator's launch latencies to rocprofv3 kernel durations.

Reference: util/tuner/GPU_Microbenchmark/ubench/system/kernel_lat (kernel
launch latency vs thread-block count) and the QV100 config's
``-gpgpu_kernel_launch_latency 5000`` / ``-gpgpu_TB_launch_latency``
(gpu-sim.cc:746-757, applied as ``kernel_launch_latency + n_blocks *
TB_launch_latency`` cycles before a kernel issues CTAs).

The correlator's hardware cycles are ``rocprofv3 duration x clock``; an empty
kernel's duration is therefore exactly the fixed cost the simulated kernel
must carry.  ``bin/ubench/ub_launch`` launches empty kernels (each right behind a ~20 us busy kernel, then synchronised) of
1..16384 workgroups; this script runs it under ``rocprofv3 --kernel-trace``
(or reads an existing run with ``-i``), fits ``duration = a + b * blocks`` on
the per-grid medians, and prints the two options in the micro-benchmark
output format the tuner reads:

    launch_latency.py -o gpurun_out/ubench/launch_rocprof   > gpurun_out/ubench/ub_launch_rocprof.log
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import subprocess
import sys
from collections import defaultdict
from typing import Dict, List, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def read_durations(run_dir: str, name_sub: str = "ub_empty_kernel") -> Dict[int, List[float]]:
    """{workgroups: [duration ns, ...]} of the empty-kernel dispatches."""
    per: Dict[int, List[float]] = defaultdict(list)
    for f in glob.glob(os.path.join(run_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if name_sub not in row.get("Kernel_Name", ""):
                    continue
                try:
                    gx = int(row["Grid_Size_X"]) // max(1, int(row["Workgroup_Size_X"]))
                    d = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                except (KeyError, ValueError, ZeroDivisionError):
                    continue
                per[gx].append(float(d))
    return dict(per)


def fit(per: Dict[int, List[float]]) -> Tuple[float, float]:
    """(a ns, b ns/workgroup) of duration = a + b * workgroups on per-grid medians."""
    xs = np.array(sorted(per), dtype=np.float64)
    ys = np.array([np.median(per[int(x)]) for x in xs])
    if len(xs) < 2:
        return float(ys[0]) if len(ys) else 0.0, 0.0
    b, a = np.polyfit(xs, ys, 1)
    return float(a), float(max(0.0, b))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-o", "--out", default=os.path.join(REPO, "gpurun_out", "ubench", "launch_rocprof"))
    ap.add_argument("-i", "--input", default="", help="existing rocprofv3 output directory (skip the run)")
    ap.add_argument("--mhz", type=float, default=0.0, help="shader clock (default: read from ub_launch)")
    ap.add_argument("--exe", default=os.path.join(REPO, "bin", "ubench", "ub_launch"))
    o = ap.parse_args(argv)
    run_dir = o.input
    mhz = o.mhz
    if not run_dir:
        run_dir = o.out
        os.makedirs(run_dir, exist_ok=True)
        cmd = ["timeout", "-k", "10", "180", "rocprofv3", "--kernel-trace", "--output-format", "csv",
               "-d", run_dir, "-o", "run", "--", o.exe]
        env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
        p = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if p.returncode != 0:
            print(p.stdout[-2000:], file=sys.stderr)
            return p.returncode
        for line in p.stdout.splitlines():
            if line.startswith("# measured_shader_mhz") and not mhz:
                mhz = float(line.split()[-1])
    mhz = mhz or 2400.0
    per = read_durations(run_dir)
    if not per:
        print("launch_latency: no ub_empty_kernel dispatches found", file=sys.stderr)
        return 1
    for nb in sorted(per):
        d = per[nb]
        print(f"empty kernel {nb:6d} workgroups: median {np.median(d):8.0f} ns  min {min(d):8.0f} ns  (n={len(d)})")
    a, b = fit(per)
    print(f"# rocprof_launch_ns {a:.1f}")
    print(f"# rocprof_per_block_ns {b:.4f}")
    have_idle = bool(read_durations(run_dir, "ub_empty_idle"))
    if not have_idle:  # older ub_launch: the isolated (after-event) launch is the only one
        print(f"-gpgpu_kernel_launch_latency {int(round(a * mhz / 1000.0))}")
        print(f"-gpgpu_TB_launch_latency {int(round(b * mhz / 1000.0))}")
    # back-to-back launches (no event / sync between): the queued cost
    q = read_durations(run_dir, "ub_empty_queued")
    if q:
        for nb in sorted(q):
            d = q[nb]
            print(f"queued empty kernel {nb:6d} workgroups: median {np.median(d):8.0f} ns  min {min(d):8.0f} ns  (n={len(d)})")
        qa, _ = fit(q)
        # reported, not applied: under rocprofv3 a queued dispatch's duration
        # also covers its wait behind the previous one (start stamps overlap
        # the previous end), so it is no per-kernel launch cost; measured on
        # MI355X: 4.7 us queued vs 3.7 us isolated vs ~2 us for a host-bound
        # launch into an idle queue (pathfinder), see profiles/ubench_mi355x
        print(f"# rocprof_queued_launch_ns {qa:.1f}")
        print(f"# queued_launch_cycles {int(round(qa * mhz / 1000.0))}")
        # a dependent kernel dispatched right behind another occupies the
        # command processor at least this long (its start stamp is the
        # previous kernel's end): the simulator's minimum queued duration
        print(f"-sim_kernel_min_cycles_queued {int(round(qa * mhz / 1000.0))}")
    # launches into an idle queue after a host gap (no event in between)
    idle = read_durations(run_dir, "ub_empty_idle")
    if idle:
        for nb in sorted(idle):
            d = idle[nb]
            print(f"idle empty kernel {nb:6d} workgroups: median {np.median(d):8.0f} ns  min {min(d):8.0f} ns  (n={len(d)})")
        ia, ib = fit(idle)
        print(f"# rocprof_idle_launch_ns {ia:.1f}")
        print(f"# rocprof_idle_per_block_ns {ib:.4f}")
        print(f"# idle_launch_cycles {int(round(ia * mhz / 1000.0))}")
        # the model's launch latency (to the first workgroup) is the idle
        # launch; a queued kernel pays the same plus the minimum duration
        # above.  Applied by the tuner (suggest_ lines): every launch
        # parameter comes from this micro-benchmark, none is fitted on the
        # suite (correlation protocol, profiles/correlation/README.md)
        il = int(round(ia * mhz / 1000.0))
        print(f"# suggested -gpgpu_kernel_launch_latency {il}")
        print(f"# suggest_gpgpu_kernel_launch_latency {il}")
        print(f"# suggest_gpgpu_kernel_launch_latency_queued {il}")
        print(f"-gpgpu_TB_launch_latency {int(round(ib * mhz / 1000.0))}")
    # the first kernel after a host-to-device copy vs the same kernel re-run
    ac = read_durations(run_dir, "ub_touch_after_copy")
    ag = read_durations(run_dir, "ub_touch_again")
    if ac and ag:
        a_med = float(np.median([x for v in ac.values() for x in v]))
        g_med = float(np.median([x for v in ag.values() for x in v]))
        print(f"# after_copy_kernel_ns {a_med:.1f}\n# same_kernel_again_ns {g_med:.1f}")
        print(f"# after_copy_extra_cycles {int(round((a_med - g_med) * mhz / 1000.0))}")
        print(f"# suggested -sim_first_kernel_latency {max(0, int(round((a_med - g_med) * mhz / 1000.0)))}")
        print(f"# suggest_sim_first_kernel_latency {max(0, int(round((a_med - g_med) * mhz / 1000.0)))}")
    # back-to-back chains: steady-state start-to-start interval and duration
    ch = chain_stats(run_dir)
    if ch:
        print(f"# chain_start_interval_ns {ch[0]:.1f}")
        print(f"# chain_duration_ns {ch[1]:.1f}")
        print(f"# chain_gap_ns {ch[2]:.1f}")
        # a host loop submitting back to back: its start-to-start interval is
        # the host's submission interval (the GPU-side queued minimum is
        # shorter), what -sim_host_launch_interval models
        print(f"# suggest_sim_host_launch_interval {int(round(ch[0] * mhz / 1000.0))}")
    return 0


def chain_stats(run_dir: str, name_sub: str = "ub_empty_chain"):
    """(median start-to-start interval, median duration, median end-to-start
    gap) over the back-to-back chain dispatches, skipping each chain's first
    four (the queue fills)."""
    rows = []
    for f in glob.glob(os.path.join(run_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if name_sub in row.get("Kernel_Name", ""):
                    rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    if len(rows) < 16:
        return None
    rows.sort()
    iv, du, gp = [], [], []
    run = 0
    for i, (s, e) in enumerate(rows):
        if i and s - rows[i - 1][1] > 20000:  # a new chain (30 us host gap)
            run = 0
        if i and run >= 4:
            iv.append(s - rows[i - 1][0])
            gp.append(s - rows[i - 1][1])
            du.append(e - s)
        run += 1
    if not iv:
        return None
    return float(np.median(iv)), float(np.median(du)), float(np.median(gp))


if __name__ == "__main__":
    sys.exit(main())
