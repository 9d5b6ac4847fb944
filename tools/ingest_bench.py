#!/usr/bin/env python3
"""Host coalescer vs the MI355X matrix-core coalescer on the synthetic suite.

For every kernel trace of the Rodinia-2.0-ft-shaped suite (plus a scaled-up
copy with --scale), runs trace.cc coalesce_kernel and
engine/ingest_mfma.hip gpu_coalesce_kernel on the same HostKernel, checks the
outputs are byte-identical and prints one JSON line with the totals.
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="GV100")
    ap.add_argument("--out", default="")
    ap.add_argument("--big", action="store_true", help="add larger instances of three generators")
    ap.add_argument("--reps", type=int, default=2, help="repeat the comparison (first pass warms caches)")
    args = ap.parse_args()
    import torch  # bind torch's HIP runtime first
    assert torch.cuda.is_available()
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    mod = _native.load(prefer_torch_runtime=True)
    cfg = presets.args_for(args.preset)
    root = tempfile.mkdtemp(prefix="ingest_")
    kl = rodinia.generate_suite(root)
    if args.big:
        # larger instances of the same generators: ingest throughput at scale
        kl["big-srad_v2"] = rodinia.write_app(os.path.join(root, "big_srad"), rodinia.srad_v2(rows=1024, cols=1024, iters=1))
        kl["big-hotspot"] = rodinia.write_app(os.path.join(root, "big_hotspot"), rodinia.hotspot(grid_n=1024, iters=1))
        kl["big-streamcluster"] = rodinia.write_app(os.path.join(root, "big_sc"),
                                                    rodinia.streamcluster(n_points=65536, launches=2))
    for _ in range(max(0, args.reps - 1)):  # warm-up passes: page-in, device buffers, code objects
        for app, path in sorted(kl.items()):
            d = os.path.dirname(path)
            for fn in sorted(os.listdir(d)):
                if fn.endswith(".asimk") or fn.endswith(".traceg"):
                    mod.ingest_compare(os.path.join(d, fn), cfg, 0)
    tot = {"kernels": 0, "insts": 0, "accs": 0, "host_s": 0.0, "device_total_s": 0.0, "device_s": 0.0,
           "smem_device": 0, "smem_host": 0, "gmem_device": 0, "gmem_host": 0, "mfma": 0, "equal": True}
    per_app = {}
    for app, path in sorted(kl.items()):
        d = os.path.dirname(path)
        a = {"host_s": 0.0, "device_total_s": 0.0, "smem_device": 0, "smem_host": 0, "gmem_device": 0, "gmem_host": 0}
        for fn in sorted(os.listdir(d)):
            if not (fn.endswith(".asimk") or fn.endswith(".traceg")):
                continue
            r = mod.ingest_compare(os.path.join(d, fn), cfg, 0)
            tot["kernels"] += 1
            tot["insts"] += r["n_insts"]
            tot["accs"] += r["n_accs"]
            tot["host_s"] += r["host_s"]
            tot["device_total_s"] += r["total_s"]
            tot["device_s"] += r["device_s"]
            for k in ("smem_device", "smem_host", "gmem_device", "gmem_host"):
                tot[k] += r[k]
                a[k] += r[k]
            tot["mfma"] += r["mfma"]
            tot["equal"] = tot["equal"] and bool(r["equal"])
            a["host_s"] += r["host_s"]
            a["device_total_s"] += r["total_s"]
        per_app[app] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in a.items()}
    tot = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in tot.items()}
    out = {"preset": args.preset, "total": tot, "apps": per_app}
    line = json.dumps(out)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
