#!/usr/bin/env python3
"""Model-regression oracle for engine refactors: simulate every suite app on
the CPU engine and record cycles, instructions and every final statistic.

    python tools/golden_stats.py --out /tmp/golden.json          # record
    python tools/golden_stats.py --check /tmp/golden.json         # compare

A refactor that must not change the model (data-structure or ordering
rewrites of csrc/model) has to reproduce the recorded file exactly.
"""
import argparse
import json
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _one(args):
    app, kl, config, extra = args
    from accel_sim_framework_distributed_amd import sim
    r = sim.simulate(kl, config, engine="cpu", extra=extra or None)
    st = {k: v for k, v in r.stats.items() if "rate" not in k and "sim_time" not in k and "silicon" not in k}
    return app, dict(cycles=r.tot_cycle, insn=r.tot_insn, stats=st)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--check")
    ap.add_argument("--config", default="QV100")
    ap.add_argument("--apps", default="all")
    ap.add_argument("--extra", default="", help="extra simulator flags, e.g. '-gpgpu_scheduler gto'")
    ap.add_argument("--trace-dir", default=os.path.join(tempfile.gettempdir(), "asim_golden_suite"))
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    apps = None if a.apps == "all" else [x if "rodinia" in x else x + "-rodinia-2.0-ft" for x in a.apps.split(",")]
    marker = os.path.join(a.trace_dir, ".complete-" + (a.apps or "all"))
    if not os.path.exists(marker):
        rodinia.generate_suite(a.trace_dir, apps)
        open(marker, "w").write("ok")
    jobs = []
    for app in sorted(os.listdir(a.trace_dir)):
        if app.startswith(".") or (apps and app not in apps):
            continue
        d = os.path.join(a.trace_dir, app)
        for args in sorted(os.listdir(d)):
            kl = os.path.join(d, args, "traces", "kernelslist.g")
            if os.path.exists(kl):
                ex = a.extra.split()
                jobs.append((app, kl, a.config, dict(zip(ex[0::2], ex[1::2])) or None))
    with ProcessPoolExecutor(a.j) as ex:
        res = dict(ex.map(_one, jobs))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)
        print(f"recorded {len(res)} apps -> {a.out}")
    if a.check:
        want = json.load(open(a.check))
        bad = 0
        for app, w in sorted(want.items()):
            g = res.get(app)
            if g is None:
                print(f"MISSING {app}")
                bad += 1
                continue
            diffs = [k for k in set(w["stats"]) | set(g["stats"]) if w["stats"].get(k) != g["stats"].get(k)]
            if g["cycles"] != w["cycles"] or g["insn"] != w["insn"] or diffs:
                bad += 1
                print(f"DIFF {app}: cycles {w['cycles']} -> {g['cycles']}, insn {w['insn']} -> {g['insn']}, "
                      f"{len(diffs)} stats differ: {sorted(diffs)[:8]}")
            else:
                print(f"ok   {app}: cycles {g['cycles']} insn {g['insn']}")
        sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
