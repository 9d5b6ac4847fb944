#!/usr/bin/env python3
"""Where a short-kernel application's time goes on the GPU engine: wall time
of the whole simulation vs the simulator's own phases, per app (GV100 preset,
the bench suite's synthetic traces).  Run under rocprofv3 --kernel-trace
--stats to split device time from host time (tools/archive/gpu_r5_overhead.sh)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from accel_sim_framework_distributed_amd import sim  # noqa: E402
from accel_sim_framework_distributed_amd.tracegen import rodinia  # noqa: E402

apps = sys.argv[1].split(",") if len(sys.argv) > 1 else ["streamcluster", "nw", "bfs"]
engine = sys.argv[2] if len(sys.argv) > 2 else "gpu"
tdir = os.path.join("/tmp", "asim_overhead_traces")
suite = rodinia.generate_suite(tdir, [a + "-rodinia-2.0-ft" for a in apps])
for a in apps:
    kl = suite[a + "-rodinia-2.0-ft"]
    for rep in range(2):
        t = time.time()
        r = sim.simulate(kl, "GV100", engine=engine)
        dt = time.time() - t
        nk = r.output.count("launching kernel name")
        print(f"{a:14s} {engine} rep {rep} wall {dt:.3f} s kernels {nk} cycles {r.tot_cycle} "
              f"insn {r.tot_insn} per-kernel {1000 * dt / max(1, nk):.1f} ms", flush=True)
