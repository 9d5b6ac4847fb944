"""Synthetic multi-rank traces of one data-parallel training step.

The reference's distributed fork traces an application whose ranks meet in
``ncclAllReduce`` calls that block the whole simulated GPU for a constant
latency (gpu-simulator/main.cc:116-122).  A real DDP step overlaps the
gradient all-reduce of layer l with the backward pass of layer l-1: the
all-reduce runs on a communication stream and waits (an event) for its
layer's gradient kernel, and the optimizer waits for the last all-reduce.
This module writes that step per rank:

    stream 1: fwd_0 .. fwd_{L-1}, bwd_{L-1} [record g_{L-1}] .. bwd_0 [record g_0],
              [wait done] optimizer
    stream 2: [wait g_{L-1}] allreduce_{L-1} .. [wait g_0] allreduce_0 [record done]

Ranks can be made unequal (``straggle``: rank r's kernels process
(1 + straggle * r / (n-1)) times the base batch shard), so the all-reduces
couple the ranks' simulated clocks mid-step: the collective starts on each
rank when its gradient is ready and finishes after the last rank joined.
Kernels are SASS-shaped (Volta / GV100 config, the bench's headline config):
a tiled GEMM-like layer kernel (global loads, shared-memory tile, barrier,
HMMA + FFMA inner loop, store) and an elementwise optimizer kernel.
"""
from __future__ import annotations

import os
from typing import List

from .builder import KernelBuilder
from .format import KernelArrays, write_kernel_binary, write_kernelslist

ACT = 0x0000720000000000   # activations
PAR = 0x0000740000000000   # parameters / gradients
LAYER = 0x0000000010000000  # 256 MB per layer


def layer_kernel(name: str, kid: int, layer: int, ctas: int, k_tiles: int, backward: bool) -> KernelArrays:
    """One GEMM-like layer pass: every CTA (128 threads) streams `k_tiles`
    tiles of A and B through shared memory and accumulates with HMMA."""
    k = KernelBuilder(name, (ctas, 1, 1), (128, 1, 1), shmem=16384, nregs=64, kid=kid)
    g = k.g
    k.op("S2R", [0])
    k.op("S2R", [1])
    k.op("IMAD", [2], [0, 1])
    a = ACT + layer * LAYER + g.cta * 65536 + g.warp * 512
    b = PAR + layer * LAYER + (g.cta % 8) * 65536 + g.warp * 512
    for t in range(k_tiles):
        k.op("LDG.E.128", [20], [2], base=a + t * 2048, stride=16)
        k.op("LDG.E.128", [24], [2], base=b + t * 2048, stride=16)
        k.op("STS.128", [], [20], base=g.warp * 512, stride=16)
        k.op("STS.128", [], [24], base=8192 + g.warp * 512, stride=16)
        k.op("BAR.SYNC")
        for j in range(4):
            k.op("LDS.128", [28], [2], base=(j * 128 + g.warp * 512) % 8192, stride=16)
            k.op("LDS.128", [32], [2], base=8192 + (j * 128) % 8192, stride=16)
            k.op("HMMA.884.F32.F32.STEP0", [40], [28, 32, 40])
            k.op("HMMA.884.F32.F32.STEP1", [42], [28, 32, 42])
            k.op("FFMA", [44], [40, 42, 44])
        k.op("BAR.SYNC")
    out = (PAR if backward else ACT) + layer * LAYER + 0x8000000 + g.cta * 65536 + g.warp * 512
    k.op("STG.E.128", [], [2, 44], base=out, stride=16)
    k.op("EXIT")
    return k.build()


def optimizer_kernel(kid: int, params: int) -> KernelArrays:
    """Elementwise SGD-with-momentum over `params` fp32 values (256 threads/CTA)."""
    ctas = max(1, params // 256)
    k = KernelBuilder("_Z13sgd_momentumPfS_S_fi", (ctas, 1, 1), (256, 1, 1), nregs=16, kid=kid)
    g = k.g
    k.op("S2R", [0])
    k.op("IMAD", [2], [0, 1])
    k.op("LDG.E", [4], [2], base=PAR + g.gtid0 * 4, stride=4)                   # weight
    k.op("LDG.E", [5], [2], base=PAR + 0x8000000 + g.gtid0 * 4, stride=4)       # gradient
    k.op("LDG.E", [6], [2], base=PAR + 0xC000000 + g.gtid0 * 4, stride=4)       # momentum
    k.op("FFMA", [6], [6, 5])
    k.op("FFMA", [4], [6, 4])
    k.op("STG.E", [], [2, 6], base=PAR + 0xC000000 + g.gtid0 * 4, stride=4)
    k.op("STG.E", [], [2, 4], base=PAR + g.gtid0 * 4, stride=4)
    k.op("EXIT")
    return k.build()


def write_dp_step(out_dir: str, rank: int = 0, nranks: int = 1, layers: int = 4, ctas: int = 80,
                  k_tiles: int = 2, grad_mb: float = 0.25, straggle: float = 0.0) -> str:
    """Write rank `rank`'s trace of one DDP step; returns its kernelslist.g.

    ``grad_mb``: gradient bucket per layer (MB, fp32) all-reduced over
    ``nranks``; ``straggle``: relative extra work of the last rank."""
    os.makedirs(out_dir, exist_ok=True)
    scale = 1.0 + (straggle * rank / (nranks - 1) if nranks > 1 else 0.0)
    my_ctas = max(1, int(round(ctas * scale)))
    count = int(grad_mb * (1 << 20) / 4)
    kernels: List[KernelArrays] = []
    cmds: List[str] = [f"ncclCommInitRank,nranks={nranks},rank={rank}"]

    def add(kern: KernelArrays) -> None:
        kernels.append(kern)
        kern.header["id"] = len(kernels)
        kern.header["stream"] = 1
        fn = f"kernel-{len(kernels)}.asimk"
        write_kernel_binary(os.path.join(out_dir, fn), kern)
        cmds.append(fn)

    for l in range(layers):
        add(layer_kernel(f"_Z11layer_fwd{l}Pf", len(kernels) + 1, l, my_ctas, k_tiles, False))
    for l in reversed(range(layers)):
        add(layer_kernel(f"_Z11layer_bwd{l}Pf", len(kernels) + 1, l, my_ctas, k_tiles, True))
        cmds.append(f"hipEventRecord,event={l + 1},stream=1")
        cmds.append(f"hipStreamWaitEvent,stream=2,event={l + 1}")
        cmds.append(f"ncclAllReduce,count={count},dtype=ncclFloat,op=ncclSum,nranks={nranks},stream=2")
    cmds.append("hipEventRecord,event=1000,stream=2")
    cmds.append("hipStreamWaitEvent,stream=1,event=1000")
    # the optimizer updates this step's parameter shard (ZeRO-1 style: 1/nranks)
    add(optimizer_kernel(len(kernels) + 1, params=max(256, int(layers * count / max(1, nranks) / 16))))
    cmds.append("ncclCommDestroy")
    return write_kernelslist(out_dir, cmds)


def write_dp_ranks(root: str, nranks: int, **kw) -> List[str]:
    """All ranks' traces under ``root/rank<r>``."""
    return [write_dp_step(os.path.join(root, f"rank{r}"), r, nranks, **kw) for r in range(nranks)]
