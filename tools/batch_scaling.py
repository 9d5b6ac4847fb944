#!/usr/bin/env python3
"""Concurrency scaling of the GPU engine: N copies of one application's
simulation (GV100 config) run side by side in one process, for N in --n.
Prints the wall time and aggregate sim KIPS per N, and the batch launcher's
counters (ASIM_GPU_BATCH=1 shares batch launches between global- / split-
state simulations; otherwise one kernel per simulation).  usage: ASIM_GPU_STATE=global python3 tools/batch_scaling.py --app hotspot --n 1,2,4"""
import argparse
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--app", default="hotspot")
    ap.add_argument("--n", default="1,2,4")
    ap.add_argument("--config", default="GV100")
    a = ap.parse_args()
    import torch
    from accel_sim_framework_distributed_amd import sim, _native
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    mod = _native.load(prefer_torch_runtime=True)
    d = tempfile.mkdtemp()
    gen = {name.split("-")[0]: g for name, (_, g) in rodinia.SUITE.items()}[a.app]
    kl = rodinia.write_app(os.path.join(d, a.app), gen())
    dev = torch.cuda.current_device()

    def one(_):
        torch.cuda.set_device(dev)
        r = sim.Simulator(a.config, kl, engine="gpu", torch_runtime=True).run()
        return r.tot_insn

    one(0)  # warm: code objects, pools
    out = []
    for n in [int(x) for x in a.n.split(",")]:
        b0 = mod.gpu_batch_stats()
        t = time.perf_counter()
        with ThreadPoolExecutor(max_workers=n) as ex:
            insn = sum(ex.map(one, range(n)))
        dt = time.perf_counter() - t
        b1 = mod.gpu_batch_stats()
        rec = {"app": a.app, "state": os.environ.get("ASIM_GPU_STATE", "split"), "n": n, "wall_s": round(dt, 3),
               "kips": round(insn / dt / 1e3, 1), "batches": b1.get("batches", 0) - b0.get("batches", 0),
               "launches": b1.get("launches", 0) - b0.get("launches", 0), "blocks_per_cu": b1.get("blocks_per_cu")}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
