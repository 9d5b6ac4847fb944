#!/usr/bin/env python3
"""Run one synthetic app on the GPU engine with the in-kernel stage profiler
(ASIM_GPU_PROFILE=1) and print wall time per epoch."""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--app", default="hotspot")
    ap.add_argument("--engine", default="gpu")
    a = ap.parse_args()
    os.environ.setdefault("ASIM_GPU_PROFILE", "1")
    import torch  # noqa: F401
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tempfile.mkdtemp()
    gen = {"vadd": lambda: [rodinia.vectoradd()]}
    for name, (_, g) in rodinia.SUITE.items():
        gen[name.split("-")[0]] = g
    gen = gen[a.app]
    kl = rodinia.write_app(os.path.join(d, a.app), gen())
    s = sim.Simulator("QV100", kl, engine=a.engine, torch_runtime=True)
    t = time.perf_counter()
    r = s.run()
    dt = time.perf_counter() - t
    print(f"{a.app}: insn={r.tot_insn} cycles={r.tot_cycle} wall={dt:.3f}s sim={r.sim_s:.3f}s "
          f"KIPS={r.tot_insn / dt / 1e3:.1f} kernels={len(r.kernels)} "
          f"epochs={sum(k.get('epochs', 0) for k in r.kernels)}", flush=True)
    del s


if __name__ == "__main__":
    main()
