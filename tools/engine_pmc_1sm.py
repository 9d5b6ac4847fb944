#!/usr/bin/env python3
"""One-SM diagnostic of the GPU engine: an app's kernels on a GV100 config
cut to ONE SM (cluster) and ONE memory channel, so the engine kernel runs two
wavefronts and rocprofv3 counters describe one SM's cycle loop without the
grid-barrier imbalance of 112 blocks.  Prints simulated cycles and the
engine's wall time; run under rocprofv3 --pmc for per-cycle instruction
counts and stall shares."""
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
    ap.add_argument("--sms", type=int, default=1)
    a = ap.parse_args()
    import torch  # noqa: F401
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tempfile.mkdtemp()
    gen = {name.split("-")[0]: g for name, (_, g) in rodinia.SUITE.items()}[a.app]
    kl = rodinia.write_app(os.path.join(d, a.app), gen())
    extra = {"-gpgpu_n_clusters": str(a.sms), "-gpgpu_n_mem": "1", "-gpgpu_n_sub_partition_per_mchannel": "2"}
    s = sim.Simulator("GV100", kl, engine=a.engine, torch_runtime=True, extra=extra)
    t = time.perf_counter()
    r = s.run()
    dt = time.perf_counter() - t
    stats = r.stats
    print(f"{a.app} sms={a.sms}: insn={r.tot_insn} cycles={r.tot_cycle} wall={dt:.3f}s sim={r.sim_s:.3f}s "
          f"epochs={sum(k.get('epochs', 0) for k in r.kernels)} "
          f"skipped={stats.get('sim_skipped_cycles', 'n/a')}", flush=True)


if __name__ == "__main__":
    main()
