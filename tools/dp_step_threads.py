#!/usr/bin/env python3
"""Host-thread scaling of the data-parallel step simulation on the CPU engine
(the node bench's critical path): generates the bench traces, then times the
dp-step at 1 / 2 / 4 threads, fastest of 2 each, in one JSON line."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    tdir = sys.argv[1] if len(sys.argv) > 1 else "/tmp/asim_dp_threads"
    kl = os.path.join(tdir, "dp-step-1", "rank0", "kernelslist.g")
    if not os.path.exists(kl):
        subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--engine", "cpu", "--apps", "dp-step",
                        "--steps", "1", "--warmup", "0", "--trace-dir", tdir], check=True, capture_output=True)
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.parallel.multi_gpu import build_args
    mod = _native.load()
    out = {}
    for th in (1, 2, 4):
        extra = {"-collective_model": "packet", "-gpgpu_concurrent_kernel_sm": "1", "-collective_mem_traffic": "1",
                 "-sim_cpu_threads": str(th)}
        best = float("inf")
        for _ in range(2):
            s = mod.Simulator(build_args("GV100", kl, "cpu", extra), False)
            t = time.perf_counter()
            assert s.run() == 0
            best = min(best, time.perf_counter() - t)
        out[th] = round(best, 4)
        print(th, out[th], flush=True)
    print(json.dumps({"dp_step_cpu_s_by_threads": out, "cpus": len(os.sched_getaffinity(0))}))


if __name__ == "__main__":
    main()
