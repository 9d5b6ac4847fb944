#!/usr/bin/env python3
"""Per-epoch cost of the packet collective's exchange primitive
(csrc/parallel/exchange.cc a2a: pinned host -> device -> all-to-all ->
host, one stream sync), timed `--iters` times through the native path.

On a 1-GPU box: a 1-rank RCCL group exchanging the words of an 8-rank epoch
(loopback, the same payload per rank), next to the same loop on gloo.  The
multi-rank RCCL number needs the 8-GPU node (the driver's SCALE run)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--shape-world", type=int, default=8)
    ap.add_argument("--out", default=None)
    ap.add_argument("--dev-bytes", type=int, default=256 << 20)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    os.environ.setdefault("ASIM_SEGV_TRACE", "1")  # native stack on a crash
    import torch
    import torch.distributed as dist
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.parallel import collectives
    PARAMS = dict(link_gbps=153.0, latency_ns=1000.0, links=7, slice_bytes=131072, max_channels=16, reduce_gbps=900.0)
    ext = _native.load_dist()
    if ext is None:
        raise SystemExit("_asim_dist not built")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    res = {}
    backends = ["gloo"] + (["nccl"] if torch.cuda.is_available() else [])
    for be in backends:
        dist.init_process_group(be, rank=0, world_size=1)
        pg = dist.distributed_c10d._get_default_group()
        dev = torch.cuda.current_device() if be == "nccl" else -1
        if be == "nccl":
            torch.cuda.set_device(dev)
        r = dict(ext.a2a_bench(pg, iters=a.iters, warm=50, device=dev, shape_world=a.shape_world))
        res[be] = r
        print(be, json.dumps(r), flush=True)
        if be == "nccl":
            # device-resident loop (linksim_dev.hip): all ranks of a shape_world-rank
            # collective on this GPU, one epoch kernel + one RCCL all-to-all
            # (1-rank loopback of every rank's slots) per epoch, no host bounce
            starts = [0] * a.shape_world
            for kind, nbytes in (("AllReduce", a.dev_bytes), ("AllToAll", a.dev_bytes)):
                ext.dev_run_local(PARAMS, kind, 16 << 20, 0, starts, dev, pg)  # warm
                d = dict(ext.dev_run_local(PARAMS, kind, nbytes, 0, starts, dev, pg, a.batch))
                t = dict(ext.dev_run_local(PARAMS, kind, nbytes, 0, starts, dev, None, a.batch))
                ref = collectives.emulate(PARAMS, kind, nbytes, starts)["finish_ps"]
                row = {"bytes": nbytes, "epochs": d["epochs"], "exchanges": d["exchanges"], "polls": d["polls"],
                       "us_per_epoch_rccl_loopback": d["us_per_epoch"], "us_per_epoch_transpose": t["us_per_epoch"],
                       "epoch_kernel_clocks_load_unpack_pack_store": [round(x) for x in t["kernel_clocks_per_launch"]],
                       "finish_equals_host_emulation": list(d["finish_ps"]) == list(ref) == list(t["finish_ps"])}
                res["device_loop_%s" % kind] = row
                print("device_loop", kind, json.dumps(row), flush=True)
        dist.destroy_process_group()
    out = {"what": "per-epoch exchange cost, 1-rank loopback of the %d-rank epoch shape" % a.shape_world,
           "path": "gloo / nccl: csrc/parallel/exchange.cc a2a (H2D async, alltoall_base, D2H async, one stream "
                   "sync); device_loop_*: linksim_dev.hip epoch kernel + RCCL all-to-all of device buffers, status "
                   "read once per batch of up to --batch epochs",
           "results": res}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
