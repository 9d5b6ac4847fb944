#!/usr/bin/env python3
"""Per-application timing of the bench suite on one engine: every Rodinia-2.0-ft
app simulated alone (wall, engine-only time, epochs, insn, cycles), then the
whole suite as bench.py runs it.  Shows where a bench step's wall time goes."""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.environ.get("ASIM_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", default="gpu")
    ap.add_argument("--config", default="QV100")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (binds torch's HIP runtime first)
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.parallel.multi_gpu import DistributedSuite
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tempfile.mkdtemp(prefix="asim_apps_")
    rodinia.generate_suite(d)
    suite = DistributedSuite(d, config=a.config, engine=a.engine)
    rows = []
    for app, kl in suite.apps:
        s = sim.Simulator(a.config, kl, engine=a.engine, torch_runtime=True)
        t = time.perf_counter()
        r = s.run()
        dt = time.perf_counter() - t
        row = dict(app=app, insn=r.tot_insn, cycles=r.tot_cycle, wall_s=round(dt, 4), sim_s=round(r.sim_s, 4),
                   kernels=len(r.kernels), kips=round(r.tot_insn / dt / 1e3, 1),
                   us_per_cycle=round(dt / max(1, r.tot_cycle) * 1e6, 3))
        rows.append(row)
        print(json.dumps(row), flush=True)
        del s
    suite.step()  # warm
    t = time.perf_counter()
    st = suite.step()
    dt = time.perf_counter() - t
    tot = dict(suite_wall_s=round(dt, 4), insn=st["insn"], cycles=st["cycles"], kips=round(st["insn"] / dt / 1e3, 1),
               concurrency=suite.concurrency(), serial_sum_s=round(sum(r["wall_s"] for r in rows), 4))
    print(json.dumps(tot), flush=True)
    if a.out:
        json.dump(dict(apps=rows, suite=tot), open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
