"""Packet-level collectives across simulated GPUs, one per rank.

Each rank runs the native ``LinkSim`` of its simulated GPU (csrc/parallel/
linksim.h): the collective is cut into RCCL-style channel/step/slice packets
on point-to-point links.  Ranks advance in lock-step epochs no longer than
the link latency (conservative PDES lookahead) and after every epoch
exchange the packets they put on the wire with ``all_to_all_single`` -- RCCL
over xGMI on MI355X (backend "nccl"), gloo on CPU.  Per epoch:

1. ``emit``: every packet whose send starts in [t, t+E) gets its arrival time;
2. header all-to-all: per-destination packet counts and each rank's total;
3. payload all-to-all (skipped when no rank sent anything): 32-byte packets;
4. ``receive`` and one all-reduce of (next event, not-done) to pick the next
   epoch start -- idle stretches are skipped, deterministically on all ranks.

The result is bit-identical to ``_asim.linksim_run_local`` with the same
arrival times, which runs every rank in one process (tests check this over
gloo with world size 2).  The reference has no counterpart: its distributed
fork charges ``-nccl_allreduce_latency`` cycles per all-reduce
(gpu-simulator/main.cc:116-122).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from .. import _native

NEVER = (1 << 64) - 1
_I64_MAX = (1 << 63) - 1


class PacketExchange:
    """Runs one collective's LinkSim epochs over a torch.distributed group."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if device is None:
            backend = dist.get_backend(group)
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.device = device
        self.stats = dict(epochs=0, packets=0, exchanges=0)

    def _a2a(self, send: "np.ndarray", out_counts: List[int], in_counts: List[int]) -> "np.ndarray":
        t = self.torch
        src = t.from_numpy(np.ascontiguousarray(send)).to(self.device)
        dst = t.empty(sum(in_counts), dtype=t.int64, device=self.device)
        self.dist.all_to_all_single(dst, src, output_split_sizes=in_counts, input_split_sizes=out_counts,
                                    group=self.group)
        self.stats["exchanges"] += 1
        return dst.cpu().numpy()

    def run(self, params: Dict, kind: str, nbytes: int, root: int, start_ps: int) -> Dict:
        mod = _native.load(prefer_torch_runtime=True)
        W, R = self.world, self.rank
        ls = mod.LinkSim(params, kind, int(nbytes), int(root), R, W, int(start_ps))
        t_dev = self.torch.tensor([min(int(start_ps), _I64_MAX)], dtype=self.torch.int64, device=self.device)
        self.dist.all_reduce(t_dev, op=self.dist.ReduceOp.MIN, group=self.group)
        t = int(t_dev.item())
        E = int(ls.epoch_ps)
        while True:
            t_end = t + E
            out = np.frombuffer(ls.emit(t_end), dtype=np.int64).reshape(-1, 4)
            dst = (out[:, 0] >> 32).astype(np.int64) if len(out) else np.zeros(0, np.int64)
            order = np.argsort(dst, kind="stable")
            counts = np.bincount(dst, minlength=W).astype(np.int64)
            # header: [packets for you, my total]
            hdr = np.stack([counts, np.full(W, len(out), np.int64)], axis=1).reshape(-1)
            rh = self._a2a(hdr, [2] * W, [2] * W).reshape(W, 2)
            in_counts = rh[:, 0].tolist()
            if int(rh[:, 1].sum()) > 0:
                payload = out[order].reshape(-1)
                inc = self._a2a(payload, (counts * 4).tolist(), [c * 4 for c in in_counts])
                if len(inc):
                    ls.receive(inc.astype(np.int64).tobytes())
                self.stats["packets"] += len(out)
            ne = ls.next_event()
            st = self.torch.tensor([min(ne, _I64_MAX), 0 if ls.done() else 1], dtype=self.torch.int64,
                                   device=self.device)
            # one all-reduce: MIN next event, MAX not-done (negated into a MIN)
            st[1] = -st[1]
            self.dist.all_reduce(st, op=self.dist.ReduceOp.MIN, group=self.group)
            gne, not_done = int(st[0].item()), -int(st[1].item())
            self.stats["epochs"] += 1
            if not not_done:
                break
            if gne >= _I64_MAX:
                raise RuntimeError("packet collective deadlocked (no rank has pending work)")
            t = max(t_end, gne)
        return dict(finish_ps=int(ls.finish_ps), channels=int(ls.channels), packets_sent=int(ls.packets_sent))


class PacketCollective:
    """Collective hook for ``Simulator.set_collective_hook`` using the packet
    model.  With more than one rank the ranks synchronise over
    torch.distributed; a collective naming a different rank count than the
    process group (or a single process) is emulated locally."""

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.ex = PacketExchange(group, device) if self.distributed else None
        self.events: List[Dict] = []

    def __call__(self, sim, desc: Dict, now: int) -> int:
        mod = _native.load(prefer_torch_runtime=True)
        params = sim.link_params()
        period = float(sim.core_period_ps)
        start = int(round(now * period))
        n = max(1, int(desc.get("nranks", 1)))
        kind, nbytes, root = desc["op"], int(desc["bytes"]), max(0, int(desc.get("root", 0)))
        if n <= 1:
            cyc, mode = 0, "single"
        elif self.distributed and n == self.ex.world:
            r = self.ex.run(params, kind, nbytes, root, start)
            cyc, mode = int(np.ceil((r["finish_ps"] - start) / period)), "rccl"
        else:
            r = mod.linksim_run_local(params, kind, nbytes, root, [0] * n)
            cyc, mode = int(np.ceil(max(r["finish_ps"]) / period)), "local"
        self.events.append(dict(op=kind, bytes=nbytes, nranks=n, now=now, cycles=cyc, mode=mode))
        return cyc


def emulate(params: Dict, kind: str, nbytes: int, starts_ps: List[int], root: int = 0) -> Dict:
    """All ranks in-process (reference for the distributed path)."""
    mod = _native.load()
    return mod.linksim_run_local(params, kind, int(nbytes), int(root), [int(s) for s in starts_ps])
