#!/usr/bin/env python3
"""How simulated cycles depend on the interconnect latency, which is also the
PDES lookahead (epoch length) of both engines.

Simulates the Rodinia-2.0-ft-shaped suite with -icnt_latency 1, 2, 4, 8 (and
16) on the CPU engine and prints / writes per-app cycles and the change
relative to latency 1 (a one-cycle crossbar, the reference's
local_interconnect default of no extra latency):

    tools/icnt_sensitivity.py [-c GV100] [-o profiles/icnt_latency_sensitivity.json]
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sweep(config="GV100", lats=(1, 2, 4, 8, 16), apps=None):
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    root = tempfile.mkdtemp(prefix="asim_icnt_")
    kls = rodinia.generate_suite(root, apps)
    out = {}
    for app, kl in kls.items():
        cyc = {}
        for L in lats:
            r = sim.simulate(kl, config, engine="cpu", extra={"-icnt_latency": str(L)})
            cyc[L] = r.tot_cycle
        out[app] = {"cycles": cyc, "pct_vs_1": {L: round(100.0 * (cyc[L] - cyc[lats[0]]) / cyc[lats[0]], 2)
                                               for L in lats}}
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-c", "--config", default="GV100")
    ap.add_argument("-o", "--out", default="")
    o = ap.parse_args()
    res = sweep(o.config)
    for app, d in res.items():
        print(f"{app:32s} " + "  ".join(f"L{L}: {c:8d} ({d['pct_vs_1'][L]:+6.2f}%)" for L, c in d["cycles"].items()))
    if o.out:
        with open(o.out, "w") as f:
            json.dump({"config": o.config, "apps": res}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
