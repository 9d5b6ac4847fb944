#!/usr/bin/env python3
"""Re-simulate captured MI355X traces on the CPU engine and correlate them
against the rocprofv3 timings of the same apps (no GPU needed).

Inputs are what tools/gpu_correlate.sh leaves behind: a traces archive or
directory (``<traces>/<app>/<args>/traces/kernelslist.g``) and the hardware
runs (``<hw>/<app>/<args>/run_<i>/``).  Used to iterate on the MI355X model
between GPU runs:

    tools/local_correlate.py -t /tmp/corr/traces -H gpurun_out/corr/hw \
        -c configs/tuned/AMD_Instinct_MI355X [-x "-opt value ..."]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import shlex
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from accel_sim_framework_distributed_amd.plotting import correlate  # noqa: E402


def sim_one(kl: str, cfg_dir: str, extra: str, exe: str = "") -> list:
    args = [exe or os.path.join(ROOT, "bin", "accel-sim.out"), "-config", os.path.join(cfg_dir, "gpgpusim.config")]
    tc = os.path.join(cfg_dir, "trace.config")
    if os.path.exists(tc):
        args += ["-config", tc]
    args += ["-trace", kl] + shlex.split(extra)
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(args, capture_output=True, text=True, env=env).stdout
    return [int(x) for x in re.findall(r"^gpu_sim_cycle = (\d+)", out, re.M)]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-t", "--traces", required=True)
    ap.add_argument("-H", "--hw", required=True)
    ap.add_argument("-c", "--config", default=os.path.join(ROOT, "configs", "tuned", "AMD_Instinct_MI355X"))
    ap.add_argument("-x", "--extra", default="", help="extra simulator options")
    ap.add_argument("--mhz", type=float, default=0.0, help="HW clock (default: the config's core clock)")
    ap.add_argument("-j", "--jobs", type=int, default=4)
    ap.add_argument("-o", "--json", default="")
    ap.add_argument("--bin", default="", help="simulator executable (default bin/accel-sim.out)")
    o = ap.parse_args(argv)
    mhz = o.mhz
    if not mhz:
        m = re.search(r"-gpgpu_clock_domains\s+([\d.]+)", open(os.path.join(o.config, "gpgpusim.config")).read())
        mhz = float(m.group(1)) if m else 2400.0
    hw = correlate.load_hw_rocprof(o.hw, burn=1)
    apps = sorted(a for a in hw if os.path.exists(os.path.join(o.traces, a, "traces", "kernelslist.g")))
    with ThreadPoolExecutor(o.jobs) as ex:
        sims = dict(zip(apps, ex.map(lambda a: sim_one(os.path.join(o.traces, a, "traces", "kernelslist.g"),
                                                        o.config, o.extra, o.bin), apps)))
    rows, errs = [], []
    for a in apps:
        ks = hw[a]
        s = sims[a]
        n = min(len(ks), len(s))
        h = sum(np.median(ks[i]["duration_ns"]) * mhz / 1000.0 for i in range(n))
        sv = float(sum(s[:n]))
        e = (sv - h) / h * 100 if h else float("nan")
        errs.append(abs(e))
        rows.append(dict(app=a, hw_cycles=h, sim_cycles=sv, err_pct=e, kernels=n))
        print(f"{a:28s} hw {h:10.0f}  sim {sv:10.0f}  err {e:+7.1f}%")
    res = dict(mae_pct=float(np.mean(errs)) if errs else None, apps=rows, config=o.config, extra=o.extra)
    print(f"cycle MAE over {len(errs)} apps: {res['mae_pct']:.2f}%")
    if o.json:
        with open(o.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
