#!/usr/bin/env python3
"""Per-epoch host overhead of the distributed packet collective, Python loop
vs the native C++ loop (csrc/parallel/exchange.cc), N gloo ranks on the CPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/exchange_overhead.py --out profiles/r4/exchange_overhead_8rank_gloo.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from accel_sim_framework_distributed_amd.parallel import collectives
    W, R = dist.get_world_size(), dist.get_rank()
    params = dict(link_gbps=153.0, latency_ns=1000.0, links=7, slice_bytes=65536, max_channels=16, reduce_gbps=900.0)
    cases = [("AllReduce", 64 << 20), ("AllGather", 32 << 20), ("ReduceScatter", 32 << 20)]
    res = {}
    for mode in ("0", "1"):
        os.environ["ASIM_NATIVE_EXCHANGE"] = mode
        best = None
        for _ in range(a.reps):
            ex = collectives.PacketExchange()
            dist.barrier()
            t = time.perf_counter()
            fin = [ex.run(params, k, b, 0, 0)["finish_ps"] for k, b in cases]
            dist.barrier()
            dt = time.perf_counter() - t
            if best is None or dt < best[0]:
                best = (dt, dict(ex.stats), fin)
        dt, st, fin = best
        res["native" if mode == "1" else "python"] = dict(wall_s=round(dt, 4), epochs=st["epochs"],
                                                          exchanges=st["exchanges"],
                                                          us_per_epoch=round(dt / max(1, st["epochs"]) * 1e6, 1),
                                                          finish_ps=fin)
    if R == 0:
        out = dict(ranks=W, backend="gloo (CPU)", cases=[f"{k} {b >> 20} MiB" for k, b in cases], **res,
                   speedup=round(res["python"]["wall_s"] / res["native"]["wall_s"], 2),
                   identical=res["python"]["finish_ps"] == res["native"]["finish_ps"])
        print(json.dumps(out))
        if a.out:
            json.dump(out, open(a.out, "w"), indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
