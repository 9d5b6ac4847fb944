"""Standalone network runs of the router model (the reference's intersim2
``booksim`` binary: ``intersim2/main.cpp`` + ``trafficmanager.cpp``).

Reads a Booksim ``.icnt`` file (topology, router pipeline, ``num_vcs``,
``vc_buf_size``, ``sw_allocator``, ``alloc_iters``, ``credit_delay``,
``internal_speedup``; the ``power_*`` per-event energies of the network
power estimate) and drives open-loop synthetic traffic through the
input-queued router model of ``csrc/model/icnt_router.h`` -- the same code
the simulator runs per epoch with ``-icnt_link_contention 2``.

    python -m accel_sim_framework_distributed_amd.icnt.booksim config.icnt \\
        --traffic uniform --rates 0.1,0.2,0.4,0.6 --packet-flits 1

prints Booksim-style ``Overall average latency`` / ``accepted rate`` lines
per injection rate (flits per node per cycle) and optionally a JSON curve.
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Dict, List

from .. import _native


def run(icnt_text: str, rate: float, traffic: str = "uniform", packet_flits: int = 1, cycles: int = 5000,
        warmup: int = 1000, seed: int = 1) -> Dict[str, float]:
    return dict(_native.load().icnt_open_loop(icnt_text, traffic, rate, packet_flits, cycles, warmup, seed))


def sweep(icnt_text: str, rates: List[float], **kw) -> List[Dict[str, float]]:
    out = []
    for r in rates:
        d = run(icnt_text, r, **kw)
        d["rate"] = r
        out.append(d)
    return out


def saturation(curve: List[Dict[str, float]], factor: float = 3.0) -> float:
    """Highest offered rate whose latency stays within `factor` x zero load."""
    ok = [c["rate"] for c in curve if c["measured_packets"] and c["avg_latency"] <= factor * c["zero_load_latency"]]
    return max(ok) if ok else 0.0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("config", help="Booksim .icnt file")
    ap.add_argument("--traffic", default="uniform",
                    help="uniform, transpose, bitcomp, bitrev, shuffle, tornado, neighbor")
    ap.add_argument("--rates", default="0.05,0.1,0.2,0.3,0.4,0.5,0.6,0.8,1.0",
                    help="offered load, flits per node per cycle (comma list)")
    ap.add_argument("--packet-flits", type=int, default=1)
    ap.add_argument("--cycles", type=int, default=5000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--json", help="write the latency / throughput curve here")
    a = ap.parse_args(argv)
    text = open(a.config).read()
    curve = sweep(text, [float(x) for x in a.rates.split(",") if x], traffic=a.traffic,
                  packet_flits=a.packet_flits, cycles=a.cycles, warmup=a.warmup, seed=a.seed)
    for c in curve:
        print(f"====== Traffic {a.traffic}, injection rate {c['rate']:.3f} ======")
        print(f"Overall average latency = {c['avg_latency']:.2f} (zero load {c['zero_load_latency']:.2f}, "
              f"max {c['max_latency']:.0f})")
        print(f"Overall average accepted rate = {c['accepted']:.4f} (offered {c['offered']:.4f}; "
              f"drain rate {c['drain_throughput']:.4f})")
        e = c["energy_pj"]
        print(f"Network power = {c['power_w']:.3f} W (energy pJ: buffer {e['buffer']:.3g}, crossbar {e['crossbar']:.3g}, "
              f"link {e['link']:.3g}, allocator {e['allocator']:.3g}, leakage {e['leakage']:.3g})")
        print(f"Packets = {c['measured_packets']} measured of {c['packets']}"
              + (f", {c['deadlocked']} deadlocked" if c["deadlocked"] else ""))
    print(f"Saturation (latency <= 3x zero load): {saturation(curve):.3f} flits/node/cycle")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"config": a.config, "traffic": a.traffic, "packet_flits": a.packet_flits, "curve": curve},
                      f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
