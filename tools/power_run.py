#!/usr/bin/env python3
"""One suite application with AccelWattch power sampling on the GPU engine
(in-kernel sampler by default): the run profiled for engine_kernel's MFMA
counters (tools/archive/gpu_r4_batch3.sh)."""
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
    ap.add_argument("--in-loop", default="1")
    a = ap.parse_args()
    import torch  # noqa: F401
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.power import xmlcfg
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tempfile.mkdtemp()
    names = {k.split("-rodinia")[0]: k for k in rodinia.SUITE}
    rodinia.generate_suite(d, [names[a.app]])
    root = os.path.join(d, names[a.app])
    kl = [os.path.join(root, x, "traces", "kernelslist.g") for x in os.listdir(root)][0]
    xml = os.path.join(d, "aw.xml")
    xmlcfg.write_xml(xml, xmlcfg.default_params("QV100"))
    args = presets.args_for("GV100", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml,
                                      "-gpgpu_runtime_stat": "200:0", "-power_report_file": os.path.join(d, "p.log"),
                                      "-power_in_loop": a.in_loop, "-sim_engine": a.engine}) + ["-trace", kl]
    mod = _native.load(prefer_torch_runtime=True)
    s = mod.Simulator(args, False)
    t = time.perf_counter()
    assert s.run() == 0
    dt = time.perf_counter() - t
    keep = [l for l in s.output.splitlines() if l.startswith(("power_in_loop", "engine_kernel_launches", "gpu_avg_power"))]
    print(f"{a.app} engine={a.engine} in_loop={a.in_loop} cycles={s.tot_cycle} wall={dt:.3f}s", *keep, flush=True)


if __name__ == "__main__":
    main()
