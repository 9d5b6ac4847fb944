#!/usr/bin/env python3
"""Collect hardware per-kernel statistics on MI355X with rocprofv3.

Reference: util/hw_stats/run_hw.py:52-183 (runs every app of the selected
suites under nvprof/nsight N times, one output directory per app/args).  Here
each run is ``rocprofv3 --kernel-trace --output-format csv`` (timestamps ->
cycles in the correlator); ``-c`` adds a separate counter pass
(``--pmc ...``) per counter group (``-c`` repeatable, ``--counter_groups``
for the correlator's set) -- counters are never combined with system/runtime
tracing, and each group stays within one pass's hardware counter limits.

Layout: ``<out>/<app>/<argfolder>/run_<i>/...kernel_trace.csv`` (and
``ctr<g>_<i>/`` per counter group), consumed by plotting/correlate.py.

    run_hw.py -B asim_hip_apps -R 4 -o hw_run/rocprof/MI355X
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys
from typing import List

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import common  # noqa: E402
    from accel_sim_framework_distributed_amd.plotting.correlate import COUNTER_GROUPS  # noqa: E402
else:
    from ..job_launching import common
    from ..plotting.correlate import COUNTER_GROUPS


def rocprof_cmd(out_dir: str, exe: List[str], counters: str = "") -> List[str]:
    cmd = ["rocprofv3"]
    if counters:
        cmd += ["--pmc"] + counters.replace(",", " ").split()
    else:
        cmd += ["--kernel-trace"]
    return cmd + ["--output-format", "csv", "-d", out_dir, "-o", "run", "--"] + exe


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-B", "--benchmark_list", required=True)
    ap.add_argument("-R", "--repeat", type=int, default=4, help="runs per app (the correlator burns the first)")
    ap.add_argument("-c", "--counters", action="append", default=[],
                    help="comma separated PMC counters for an extra pass (repeatable: one pass each)")
    ap.add_argument("--counter_repeat", type=int, default=1, help="runs per counter pass (counts are deterministic)")
    ap.add_argument("--counter_groups", action="store_true",
                    help="add the correlator's counter passes (plotting/correlate.py COUNTER_GROUPS)")
    ap.add_argument("-o", "--out", default=os.path.join(common.REPO_ROOT, "hw_run", "rocprof", "MI355X"))
    ap.add_argument("-t", "--timeout", type=int, default=300, help="seconds per run")
    ap.add_argument("-n", "--dry_run", action="store_true")
    o = ap.parse_args(argv)
    reg = common.Registry()
    out = os.path.abspath(o.out)
    groups = list(o.counters)
    if o.counter_groups:
        groups += COUNTER_GROUPS
    env = dict(os.environ)
    env.pop("ASIM_TRACE_DIR", None)  # time the plain build, never the traced one
    env.setdefault("TMPDIR", "/tmp")
    for exec_dir, data_dir, app, args_list in reg.benchmarks(o.benchmark_list.split(",")):
        exe_path = os.path.join(os.path.expandvars(exec_dir) or ".", app)
        if not os.path.isabs(exe_path):
            exe_path = os.path.join(common.REPO_ROOT, exe_path)
        for a in args_list:
            args = a.get("args")
            argv_app = [exe_path] + (shlex.split(str(args)) if args else [])
            base = os.path.join(out, app, common.argfoldername(args))
            passes = [("run", "")] + [(f"ctr{g}", c) for g, c in enumerate(groups)]
            for tag, ctr in passes:
                for r in range(o.repeat if not ctr else o.counter_repeat):
                    d = os.path.join(base, f"{tag}_{r}")
                    cmd = ["timeout", "-k", "10", str(o.timeout)] + rocprof_cmd(d, argv_app, ctr)
                    print(" ".join(shlex.quote(c) for c in cmd), flush=True)
                    if o.dry_run:
                        continue
                    os.makedirs(d, exist_ok=True)
                    rc = subprocess.call(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL)
                    if rc != 0:
                        print(f"run_hw: {app} failed (rc={rc}); stopping", file=sys.stderr)
                        return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
