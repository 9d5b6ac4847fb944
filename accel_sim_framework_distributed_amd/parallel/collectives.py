"""Packet-level collectives across simulated GPUs, one per rank.

Each rank runs the native ``LinkSim`` of its simulated GPU (csrc/parallel/
linksim.h): the collective is cut into RCCL-style channel/step/slice packets
on point-to-point links.  Ranks advance in lock-step epochs no longer than
the link latency (conservative PDES lookahead) and after every epoch
exchange the packets they put on the wire with ONE fixed-size
``all_to_all_single`` -- RCCL over xGMI on MI355X (backend "nccl"), gloo on
CPU.  Per epoch:

1. ``emit``: every packet whose send starts in [t, t+E) gets its arrival time;
2. one all-to-all of a fixed slot per destination: a header (packets for you,
   my largest per-destination count, my next event and not-done flag as of
   the previous epoch, the earliest arrival among the packets I send now)
   followed by up to K packets; only if some rank had more than K for one
   destination (every rank sees that in the headers) a second, variable-size
   all-to-all carries the rest;
3. ``receive``, sources in rank order, each in emission order.

Steps 1-3 are native (``LinkSim.pack_epoch`` writes the packets straight into
the pinned send buffer, ``unpack_epoch`` delivers the received slots), so
the per-epoch host work is two calls around the all-to-all.

The next epoch starts at max(t+E, G), G = the minimum over ranks of the
previous next events and of this epoch's earliest arrivals: every event a
rank can have after this epoch is one of its earlier pending sends or is
caused by a packet exchanged now, so nothing happens before G.  The flags
and next events travel one epoch late, so the ranks stop one epoch after the
last is done; there is no separate all-reduce and no extra host sync.

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
        self._buf: Dict = {}

    def _bufs(self, n_out: int, n_in: int, tag: str = ""):
        """Exchange buffers reused across epochs: on a GPU backend a pinned
        host staging pair plus the device pair (one async H2D / D2H copy
        each way, no allocation per epoch); on the CPU the tensors
        themselves."""
        key = (tag, n_out, n_in)
        b = self._buf.get(key)
        if b is None:
            t = self.torch
            if self.device.type == "cpu":
                b = (None, t.empty(n_out, dtype=t.int64), t.empty(n_in, dtype=t.int64), None)
            else:
                b = (t.empty(n_out, dtype=t.int64, pin_memory=True), t.empty(n_out, dtype=t.int64, device=self.device),
                     t.empty(n_in, dtype=t.int64, device=self.device), t.empty(n_in, dtype=t.int64, pin_memory=True))
            if len(self._buf) > 16:
                self._buf.clear()
            self._buf[key] = b
        return b

    def _a2a(self, send: "np.ndarray", out_counts: List[int], in_counts: List[int]) -> "np.ndarray":
        n_out, n_in = int(sum(out_counts)), int(sum(in_counts))
        h_src, src, dst, h_dst = self._bufs(n_out, n_in)
        if h_src is None:
            src.numpy()[:] = send
        else:
            h_src.numpy()[:] = send
            src.copy_(h_src, non_blocking=True)
        self.dist.all_to_all_single(dst, src, output_split_sizes=in_counts, input_split_sizes=out_counts,
                                    group=self.group)
        self.stats["exchanges"] += 1
        if h_dst is None:
            return dst.numpy().copy()
        h_dst.copy_(dst, non_blocking=True)
        self.torch.cuda.current_stream().synchronize()
        return h_dst.numpy().copy()

    def _a2a_fixed(self, ls, t_end: int, ann_next: int, ann_busy: int, n: int):
        """The fixed-slot all-to-all of one epoch: LinkSim packs this rank's
        packets straight into the (pinned) send buffer; returns the received
        slots (a view, valid until the next exchange) and the overflow."""
        h_src, src, dst, h_dst = self._bufs(n, n, "fixed")  # never shared with the overflow exchange
        send = (src if h_src is None else h_src).numpy()
        extra, extra_words, npk, _ = ls.pack_epoch(t_end, self.K, self.HDR, ann_next, ann_busy, send)
        if h_src is not None:
            src.copy_(h_src, non_blocking=True)
        W = self.world
        self.dist.all_to_all_single(dst, src, output_split_sizes=[n // W] * W, input_split_sizes=[n // W] * W,
                                    group=self.group)
        self.stats["exchanges"] += 1
        if h_dst is None:
            return dst.numpy(), extra, extra_words, npk
        h_dst.copy_(dst, non_blocking=True)
        self.torch.cuda.current_stream().synchronize()
        return h_dst.numpy(), extra, extra_words, npk

    K = 8       # packet slots per destination in the fixed exchange
    HDR = 8     # header words per destination slot

    def run(self, params: Dict, kind: str, nbytes: int, root: int, start_ps: int) -> Dict:
        """One collective.  The epoch loop runs natively (csrc/parallel/
        exchange.cc over the group's c10d ProcessGroup, GIL released) unless
        ``ASIM_NATIVE_EXCHANGE=0`` or the extension is not built; on a GPU
        backend it is device-resident (csrc/parallel/linksim_dev.hip: the
        LinkSim state in HBM, one epoch kernel and one RCCL all-to-all of device
        buffers per epoch, status read every few epochs) unless
        ``ASIM_DEVICE_EXCHANGE=0``.  All loops implement the same protocol and
        give identical results."""
        import os
        dist_ext = _native.load_dist() if os.environ.get("ASIM_NATIVE_EXCHANGE", "1") != "0" else None
        if dist_ext is not None:
            pg = self.group if self.group is not None else self.dist.distributed_c10d._get_default_group()
            dev = self.device.index if self.device.type == "cuda" else -1
            if dev is None:
                dev = self.torch.cuda.current_device()
            pr = {k: v for k, v in params.items()}
            if dev >= 0 and os.environ.get("ASIM_DEVICE_EXCHANGE", "1") != "0":
                # device-resident loop: LinkSim state in HBM, one epoch kernel +
                # one RCCL all-to-all of device buffers per epoch, no host bounce
                r = dist_ext.exchange_run_device(pg, pr, kind, int(nbytes), int(root), int(start_ps), int(dev),
                                                 int(os.environ.get("ASIM_DEVICE_EXCHANGE_BATCH", "16")))
                self.stats["device_loop"] = True
                self.stats["polls"] = self.stats.get("polls", 0) + int(r["polls"])
            else:
                r = dist_ext.exchange_run(pg, pr, kind, int(nbytes), int(root), int(start_ps), int(dev))
            for k in ("epochs", "packets", "exchanges"):
                self.stats[k] += int(r[k])
            self.stats["native_loop_s"] = self.stats.get("native_loop_s", 0.0) + float(r["loop_s"])
            self.stats["native"] = True
            return dict(finish_ps=int(r["finish_ps"]), channels=int(r["channels"]),
                        packets_sent=int(r["packets_sent"]))
        mod = _native.load(prefer_torch_runtime=True)
        W, R, K, H = self.world, self.rank, self.K, self.HDR
        ls = mod.LinkSim(params, kind, int(nbytes), int(root), R, W, int(start_ps))
        t_dev = self.torch.tensor([min(int(start_ps), _I64_MAX)], dtype=self.torch.int64, device=self.device)
        self.dist.all_reduce(t_dev, op=self.dist.ReduceOp.MIN, group=self.group)
        t = int(t_dev.item())
        E = int(ls.epoch_ps)
        slot = H + 4 * K
        # state announced in the next exchange: as of the end of the previous epoch
        ann_next = min(int(ls.next_event()), _I64_MAX)
        ann_busy = 0 if ls.done() else 1
        none = np.zeros(0, np.int64)
        while True:
            t_end = t + E
            # emit + pack (native), one fixed all-to-all
            recv, extra, extra_words, npk = self._a2a_fixed(ls, t_end, ann_next, ann_busy, W * slot)
            hdr = recv.reshape(W, slot)
            inc = none
            if int(hdr[:, 1].max()) > K:
                # some rank sent more than K packets to one destination: the rest
                extra_in = [4 * max(0, int(c) - K) for c in hdr[:, 0]]
                inc = self._a2a(extra, [int(w) for w in extra_words], extra_in)
            # deliver in source order (native); flags / next events of every rank
            any_busy, g = ls.unpack_epoch(recv, K, H, inc)
            self.stats["packets"] += int(npk)
            self.stats["epochs"] += 1
            if not any_busy:
                # every rank was done before this epoch: nothing was sent in it
                break
            ann_next = min(int(ls.next_event()), _I64_MAX)
            ann_busy = 0 if ls.done() else 1
            if g >= _I64_MAX:
                # no pending send anywhere and nothing on the wire, yet a rank is not done
                raise RuntimeError("packet collective deadlocked (no rank has pending work)")
            t = max(t_end, int(g))
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


class LocalRanks:
    """All ranks in ONE process (threads), coupled like the distributed path:
    ``hook(r)`` is rank r's collective hook.  At each collective every rank
    deposits its start time and waits for the others; the packet link model
    then runs once over all ranks' start times (``linksim_run_local``) and
    each rank is charged its own finish - start.  This is the oracle the
    RCCL / gloo path (PacketCollective over PacketExchange) must match bit
    for bit, collectives overlapping compute included.  Usage:
    ``sim_r.set_collective_hook(ranks.hook(r, sim_r))``."""

    def __init__(self, nranks: int):
        import threading
        self.n = nranks
        self.lock = threading.Lock()
        self.barrier = threading.Barrier(nranks, timeout=600)
        self.starts: List[int] = [0] * nranks
        self.result: Optional[Dict] = None
        self.events: List[List[Dict]] = [[] for _ in range(nranks)]

    def hook(self, rank: int, sim):
        def call(desc: Dict, now: int) -> int:
            period = float(sim.core_period_ps)
            start = int(round(now * period))
            n = max(1, int(desc.get("nranks", 1)))
            if n != self.n:
                raise RuntimeError(f"collective over {n} ranks in a {self.n}-rank emulation")
            kind, nbytes, root = desc["op"], int(desc["bytes"]), max(0, int(desc.get("root", 0)))
            self.starts[rank] = start
            if self.barrier.wait() == 0:
                mod = _native.load()
                self.result = mod.linksim_run_local(sim.link_params(), kind, nbytes, root, list(self.starts))
            self.barrier.wait()
            fin = int(self.result["finish_ps"][rank])
            cyc = int(np.ceil((fin - start) / period))
            self.events[rank].append(dict(op=kind, bytes=nbytes, nranks=n, now=now, cycles=cyc, mode="local-ranks"))
            self.barrier.wait()  # every rank read the result before the next collective overwrites it
            return cyc
        return call


def emulate(params: Dict, kind: str, nbytes: int, starts_ps: List[int], root: int = 0) -> Dict:
    """All ranks in-process (reference for the distributed path)."""
    mod = _native.load()
    return mod.linksim_run_local(params, kind, int(nbytes), int(root), [int(s) for s in starts_ps])
