#!/usr/bin/env python3
"""Statistics-archive regression gate of the short CI run (travis.sh).

The reference's CI archives get_stats output per build and correlates it
(Jenkinsfile:54-91: get_stats -> merge-stats into a statistics archive ->
plot-correlation against hardware).  Here the archive is a committed flat CSV
in the correlator's hardware format (app,args,kernel,instance,duration_ns,
thread_insts,...), so the same file drives util/plotting/plot-correlation.py -F
and this exact per-kernel gate:

    tools/ci_regress.py --stats per_kernel.csv --record ci/golden.csv --clock_mhz 1132
    tools/ci_regress.py --stats per_kernel.csv --check  ci/golden.csv [--tolerance 0]

--check exits 1 if any kernel's cycles or instructions moved by more than
--tolerance percent (0 = bit-exact), or if kernels appeared / disappeared.
"""
from __future__ import annotations

import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from accel_sim_framework_distributed_amd.job_launching import get_stats  # noqa: E402

S_CYC = r"gpu_sim_cycle\s*=\s*(.*)"
S_INSN = r"gpu_sim_insn\s*=\s*(.*)"
S_WINSN = r"gpgpu_n_tot_w_icount\s*=\s*(.*)"


def per_kernel(stats_csv: str, config: str | None):
    """{(app, args): [(kernel, cycles, insn)] in launch order} for one config."""
    blocks = get_stats.parse_csv_blocks(open(stats_csv).read())
    cyc, ins = blocks.get(S_CYC, {}), blocks.get(S_INSN, {})
    out = {}
    for row, vals in cyc.items():
        cfg = config or next(iter(vals))
        if cfg not in vals or not vals[cfg]:
            continue
        app_args, _, kern = row.partition("--")
        app, _, args = app_args.partition("/")
        out.setdefault((app, args), []).append((kern, int(float(vals[cfg])),
                                                int(float(ins.get(row, {}).get(cfg, 0) or 0))))
    return out


def record(sim, path: str, mhz: float) -> None:
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["app", "args", "kernel", "instance", "duration_ns", "thread_insts", "cycles"])
        for (app, args), ks in sorted(sim.items()):
            for i, (k, c, n) in enumerate(ks):
                w.writerow([app, args, k.rsplit("--", 1)[0], i, f"{c * 1000.0 / mhz:.3f}", n, c])


def load_golden(path: str):
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault((r["app"], r["args"]), []).append((r["kernel"], int(r["cycles"]), int(r["thread_insts"])))
    return out


def check(sim, gold, tol_pct: float, subset: bool = False) -> int:
    bad = 0
    errs = []
    keys = set(sim) if subset else set(sim) | set(gold)
    for key in sorted(keys):
        s, g = sim.get(key, []), gold.get(key, [])
        if len(s) != len(g):
            print(f"FAIL {key[0]}: {len(s)} kernels simulated, {len(g)} in the archive")
            bad += 1
            continue
        for i, ((_, sc, sn), (gk, gc, gn)) in enumerate(zip(s, g)):
            e = abs(sc - gc) / max(1, gc) * 100.0
            errs.append(e)
            if e > tol_pct or (tol_pct == 0 and sn != gn):
                print(f"FAIL {key[0]} kernel {i} ({gk}): cycles {sc} vs {gc} ({e:.2f} %), insn {sn} vs {gn}")
                bad += 1
    n = len(errs)
    mae = sum(errs) / n if n else 0.0
    print(f"ci_regress: {len(sim)} apps, {n} kernels, cycle MAE vs archive {mae:.3f} %, {bad} failures")
    return 1 if bad else 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--stats", required=True, help="get_stats.py -k -K output")
    ap.add_argument("--config", default=None, help="config column (default: the first)")
    ap.add_argument("--record", default="")
    ap.add_argument("--check", default="")
    ap.add_argument("--tolerance", type=float, default=0.0, help="allowed per-kernel cycle drift, percent")
    ap.add_argument("--clock_mhz", type=float, default=1132.0)
    ap.add_argument("--subset", action="store_true", help="check only the simulated apps (a partial CI run)")
    a = ap.parse_args(argv)
    sim = per_kernel(a.stats, a.config)
    if not sim:
        print("ci_regress: no simulated kernels in", a.stats)
        return 1
    if a.record:
        record(sim, a.record, a.clock_mhz)
        print(f"ci_regress: archived {sum(len(v) for v in sim.values())} kernels of {len(sim)} apps to {a.record}")
    if a.check:
        return check(sim, load_golden(a.check), a.tolerance, a.subset)
    return 0


if __name__ == "__main__":
    sys.exit(main())
