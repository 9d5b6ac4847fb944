"""Synthetic Rodinia-2.0-ft-shaped traces (the north-star workload).

No NVIDIA GPU, CUDA toolchain or pre-recorded traces are available, so each
application of the suite (reference util/job_launching/apps/define-all-apps.yml:13-50,
kmeans disabled like the reference) is reproduced as a synthetic SASS trace
with the same kernel structure: launch sequence, grid/block shapes, shared
memory use, barrier placement, loop structure, instruction mix and memory
access patterns (coalesced streams, stencils, irregular gathers).  Traces are
deterministic (seeded) and written in the binary ``.asimk`` format plus a
reference-compatible ``kernelslist.g``.
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Tuple

import numpy as np

from .builder import KernelBuilder
from .format import KernelArrays, write_kernel_binary, write_kernel_text, write_kernelslist

GB = 0x0000700000000000  # first device buffer
BUF = 0x10000000         # 256 MB between buffers


def buf(i: int) -> int:
    return GB + i * BUF


def _prologue(k: KernelBuilder, n_idx: int = 3) -> None:
    k.op("S2R", [0])
    k.op("S2R", [1])
    k.op("IMAD", [2], [0, 1])
    for i in range(n_idx - 1):
        k.op("IMAD.WIDE", [10 + i], [2, 3])


def _epilogue(k: KernelBuilder) -> None:
    k.op("EXIT")


# ----------------------------------------------------------------------------
def vectoradd(n: int = 100000, block: int = 1024, kid: int = 1) -> KernelArrays:
    """nvbit test-apps/vectoradd: c[i] = a[i] + b[i] (doubles), n=100000."""
    grid = -(-n // block)
    k = KernelBuilder("_Z6vecAddPdS_S_i", (grid, 1, 1), (block, 1, 1), nregs=16, kid=kid)
    g = k.g
    tid = g.cta * block + g.tid0
    live = np.clip(n - tid, 0, 32)
    mask = ((np.uint64(1) << live.astype(np.uint64)) - np.uint64(1)).astype(np.uint64)
    mask = np.where(live >= 32, np.uint64(0xFFFFFFFF), mask)
    _prologue(k, 4)
    k.op("ISETP", [20], [2])
    k.op("LDG.E.64", [4], [10], base=buf(0) + tid * 8, stride=8, mask=mask)
    k.op("LDG.E.64", [6], [11], base=buf(1) + tid * 8, stride=8, mask=mask)
    k.op("DADD", [8], [4, 6], mask=mask)
    k.op("STG.E.64", [], [12, 8], base=buf(2) + tid * 8, stride=8, mask=mask)
    _epilogue(k)
    return k.build()


# ----------------------------------------------------------------------------
def backprop(n_in: int = 4096, kid0: int = 1) -> List[KernelArrays]:
    """bpnn_layerforward_CUDA + bpnn_adjust_weights_cuda, 16x16 blocks."""
    hid = 16
    grid = (1, n_in // 16, 1)
    out = []
    # layer forward: load input & weights to shared, log2(16)=4 reduction steps
    k = KernelBuilder("_Z22bpnn_layerforward_CUDAPfS_S_S_ii", grid, (16, 16, 1), shmem=16 * 4 + 16 * 16 * 4,
                      nregs=20, kid=kid0)
    g = k.g
    row = g.cy * 16 + g.warp * 2  # each warp covers 2 rows of 16 threads
    _prologue(k, 3)
    k.op("LDG.E", [4], [10], base=buf(0) + (g.cy * 16) * 4, stride=0)
    k.op("STS", [], [4], base=g.warp * 0, stride=0)
    k.op("BAR.SYNC")
    k.op("LDG.E", [5], [11], base=buf(1) + (row * (hid + 1)) * 4, stride=4)
    k.op("STS", [], [5], base=64 + g.warp * 128, stride=4)
    k.op("BAR.SYNC")
    k.op("LDS", [6], [2], base=64 + g.warp * 128, stride=4)
    k.op("LDS", [7], [2], base=0, stride=0)
    k.op("FMUL", [6], [6, 7])
    k.op("STS", [], [6], base=64 + g.warp * 128, stride=4)
    k.op("BAR.SYNC")
    for step in range(4):
        p = 1 << (step + 1)
        k.op("ISETP", [20], [2])
        k.op("LDS", [8], [2], base=64 + g.warp * 128, stride=4 * p)
        k.op("LDS", [9], [2], base=64 + g.warp * 128 + 4 * (p // 2), stride=4 * p)
        k.op("FADD", [8], [8, 9])
        k.op("STS", [], [8], base=64 + g.warp * 128, stride=4 * p)
        k.op("BAR.SYNC")
    k.op("LDS", [6], [2], base=64 + g.warp * 128, stride=4)
    k.op("STG.E", [], [12, 6], base=buf(2) + (g.cy * hid + g.warp * 2) * 4, stride=4)
    _epilogue(k)
    out.append(k.build())
    # adjust weights
    k = KernelBuilder("_Z24bpnn_adjust_weights_cudaPfiS_iS_S_", grid, (16, 16, 1), nregs=24, kid=kid0 + 1)
    g = k.g
    row = g.cy * 16 + g.warp * 2
    _prologue(k, 4)
    k.op("LDG.E", [4], [10], base=buf(3) + g.warp * 0, stride=4)            # delta
    k.op("LDG.E", [5], [11], base=buf(0) + row * 4, stride=0)               # ly
    k.op("LDG.E", [6], [12], base=buf(4) + (row * (hid + 1)) * 4, stride=4)  # oldw
    k.op("FMUL", [7], [4, 5])
    k.op("FMUL", [8], [6, 5])
    k.op("FFMA", [7], [7, 8, 4])
    k.op("LDG.E", [9], [12], base=buf(1) + (row * (hid + 1)) * 4, stride=4)  # w
    k.op("FADD", [9], [9, 7])
    k.op("STG.E", [], [12, 9], base=buf(1) + (row * (hid + 1)) * 4, stride=4)
    k.op("STG.E", [], [12, 7], base=buf(4) + (row * (hid + 1)) * 4, stride=4)
    k.op("BAR.SYNC")
    k.op("ISETP", [20], [2])
    k.op("LDG.E", [4], [10], base=buf(3), stride=4, mask=np.where(g.cy == 0, 0xFFFF, 0))
    k.op("FFMA", [7], [4, 5, 6], mask=np.where(g.cy == 0, 0xFFFF, 0))
    k.op("STG.E", [], [12, 7], base=buf(1), stride=4, mask=np.where(g.cy == 0, 0xFFFF, 0))
    _epilogue(k)
    out.append(k.build())
    return out


# ----------------------------------------------------------------------------
def bfs(n_nodes: int = 4096, avg_deg: int = 6, levels: int = 10, seed: int = 1, kid0: int = 1) -> List[KernelArrays]:
    """Kernel (frontier expansion, irregular gathers) + Kernel2 (mask update) per level."""
    rng = np.random.default_rng(seed)
    block = 512
    grid = (-(-n_nodes // block), 1, 1)
    out = []
    kid = kid0
    frontier_frac = [0.002, 0.01, 0.05, 0.15, 0.3, 0.25, 0.15, 0.06, 0.02, 0.005]
    for lvl in range(levels):
        frac = frontier_frac[lvl % len(frontier_frac)]
        k = KernelBuilder("_Z6KernelP4NodePiPbS2_S1_S2_i", grid, (block, 1, 1), nregs=18, kid=kid, seed=seed + lvl)
        kid += 1
        g = k.g
        tid = g.cta * block + g.tid0
        _prologue(k, 2)
        k.op("ISETP", [20], [2])
        k.op("LDG.E.CONSTANT", [4], [10], base=buf(2) + tid, stride=1)  # graph_mask (bytes)
        # active lanes: nodes in the frontier
        act = rng.random((g.nwarps, 32)) < frac
        amask = np.packbits(act[:, ::-1], axis=1, bitorder="big").view(">u4").reshape(-1).astype(np.uint64)
        k.op("ISETP", [21], [4])
        k.op("BSSY", [], [], mask=amask)
        k.op("LDG.E.64", [6], [10], base=buf(0) + tid * 8, stride=8, mask=amask)  # node start/len
        k.op("STG.E", [], [10], base=buf(2) + tid, stride=1, mask=amask)
        max_deg = 2 * avg_deg
        for e in range(max_deg):
            emask = amask & np.where(rng.random(g.nwarps) < (1.0 - e / max_deg), np.uint64(0xFFFFFFFF), np.uint64(0))
            edges = rng.integers(0, n_nodes * avg_deg, size=(g.nwarps, 32))
            nbr = rng.integers(0, n_nodes, size=(g.nwarps, 32))
            k.op("IADD3", [8], [6, 7], mask=emask)
            k.op("LDG.E", [9], [8], addrs=buf(1) + edges * 4, mask=emask)          # edge list
            k.op("LDG.E.CONSTANT", [11], [9], addrs=buf(3) + nbr, mask=emask)     # visited
            k.op("ISETP", [22], [11], mask=emask)
            k.op("LDG.E", [12], [6], base=buf(4) + tid * 4, stride=4, mask=emask)  # cost[tid]
            k.op("IADD3", [12], [12], mask=emask)
            k.op("STG.E", [], [9, 12], addrs=buf(4) + nbr * 4, mask=emask)         # cost[id]
            k.op("STG.E", [], [9], addrs=buf(5) + nbr, mask=emask)                 # updating mask
            k.op("BRA", [], [22], mask=emask)
        k.op("BSYNC", [], [])
        _epilogue(k)
        out.append(k.build())
        # Kernel2: update masks
        k = KernelBuilder("_Z7Kernel2PbS_S_S_i", grid, (block, 1, 1), nregs=12, kid=kid)
        kid += 1
        g = k.g
        tid = g.cta * block + g.tid0
        _prologue(k, 2)
        k.op("ISETP", [20], [2])
        k.op("LDG.E.CONSTANT", [4], [10], base=buf(5) + tid, stride=1)
        k.op("ISETP", [21], [4])
        act = rng.random((g.nwarps, 32)) < frac * 1.5
        amask = np.packbits(act[:, ::-1], axis=1, bitorder="big").view(">u4").reshape(-1).astype(np.uint64)
        k.op("STG.E", [], [10], base=buf(2) + tid, stride=1, mask=amask)
        k.op("STG.E", [], [10], base=buf(3) + tid, stride=1, mask=amask)
        k.op("STG.E", [], [10], base=buf(6), stride=0, mask=amask & np.uint64(1))
        k.op("STG.E", [], [10], base=buf(5) + tid, stride=1, mask=amask)
        _epilogue(k)
        out.append(k.build())
    return out


# ----------------------------------------------------------------------------
def hotspot(grid_n: int = 512, pyramid: int = 2, iters: int = 6, kid0: int = 1) -> List[KernelArrays]:
    """calculate_temp: 16x16 tiles with halo, `pyramid` steps per launch."""
    bs = 16
    small = bs - 2 * pyramid
    blocks = -(-grid_n // small)
    out = []
    for it in range(max(1, iters // pyramid)):
        k = KernelBuilder("_Z14calculate_tempiPfS_S_iiiiffffff", (blocks, blocks, 1), (bs, bs, 1),
                          shmem=3 * bs * bs * 4, nregs=38, kid=kid0 + it)
        g = k.g
        row0 = g.cy * small - pyramid + g.warp * 2
        col0 = g.cx * small - pyramid
        gaddr = (np.clip(row0, 0, grid_n - 1) * grid_n + np.clip(col0, 0, grid_n - 16)) * 4
        _prologue(k, 3)
        for _ in range(6):
            k.op("IMAD", [5], [0, 1])
        k.op("ISETP", [20], [2])
        k.op("LDG.E", [6], [10], base=buf(0) + gaddr, stride=4)   # power
        k.op("LDG.E", [7], [11], base=buf(1) + gaddr, stride=4)   # temp_src
        k.op("STS", [], [6], base=g.warp * 128, stride=4)
        k.op("STS", [], [7], base=1024 + g.warp * 128, stride=4)
        k.op("BAR.SYNC")
        for p in range(pyramid):
            k.op("ISETP", [21], [2])
            for nb in range(5):
                k.op("LDS", [8 + nb], [2], base=1024 + g.warp * 128 + ((nb % 3) - 1) * 4, stride=4)
            k.op("LDS", [13], [2], base=g.warp * 128, stride=4)
            k.op("FADD", [14], [9, 10])
            k.op("FFMA", [14], [8, 14, 15])
            k.op("FADD", [16], [11, 12])
            k.op("FFMA", [16], [8, 16, 15])
            k.op("FFMA", [14], [13, 14, 16])
            k.op("FFMA", [14], [14, 17, 8])
            k.op("FSETP", [22], [14])
            k.op("BAR.SYNC")
            k.op("STS", [], [14], base=1024 + g.warp * 128, stride=4)
            k.op("BAR.SYNC")
        k.op("STG.E", [], [12, 14], base=buf(2) + gaddr, stride=4)
        _epilogue(k)
        out.append(k.build())
    return out


# ----------------------------------------------------------------------------
def heartwall(n_points: int = 51, kid0: int = 1, scale: float = 1.0, alu_per_iter: int = 0) -> List[KernelArrays]:
    """One long kernel: template matching with big ALU loops (1 frame).

    `alu_per_iter` extra independent FFMAs per loop iteration (0: the suite's
    shape, 2 global loads per 6 ALU ops; the gfx950 heartwall's measured mix
    is ~10 VALU per global load, profiles/isatrace/heartwall.verify.txt; see
    profiles/heartwall_parity.md)."""
    block = 512
    k = KernelBuilder("_Z6kernelv", (n_points, 1, 1), (block, 1, 1), shmem=4 * 1024, nregs=56, kid=kid0)
    g = k.g
    _prologue(k, 3)
    iters = int(10 * scale)
    for it in range(iters):
        off = (g.cta * 65536 + g.warp * 4096 + it * 128)
        k.op("LDG.E", [6], [10], base=buf(0) + off, stride=4)
        k.op("LDG.E", [7], [11], base=buf(1) + off, stride=4)
        for j in range(alu_per_iter):
            r = 24 + (j % 8)
            k.op("FFMA", [r], [r, 3, r])
        k.op("IMAD", [8], [2, 3])
        k.op("FADD", [9], [6, 7])
        k.op("FMUL", [9], [9, 9])
        k.op("FFMA", [12], [9, 6, 12])
        k.op("ISETP", [20], [8])
        k.op("STS", [], [12], base=g.warp * 128, stride=4)
        k.op("BAR.SYNC")
        k.op("LDS", [13], [2], base=g.warp * 128, stride=4)
        k.op("FFMA", [14], [13, 13, 14])
        k.op("BRA", [], [20])
    k.op("MUFU.SQRT", [15], [14])
    k.op("MUFU.RCP", [16], [15])
    k.op("FMUL", [17], [16, 12])
    k.op("STG.E", [], [10, 17], base=buf(2) + g.cta * 4096 + g.warp * 128, stride=4)
    _epilogue(k)
    return [k.build()]


# ----------------------------------------------------------------------------
def lud(n: int = 64, kid0: int = 1) -> List[KernelArrays]:
    """lud_diagonal / lud_perimeter / lud_internal per 16x16 block step."""
    bs = 16
    out = []
    kid = kid0
    steps = n // bs
    for s in range(steps):
        # diagonal: 1 block of 16 threads, long sequential inner loop
        k = KernelBuilder("_Z12lud_diagonalPfii", (1, 1, 1), (bs, 1, 1), shmem=bs * bs * 4, nregs=24, kid=kid)
        kid += 1
        _prologue(k, 2)
        for i in range(bs):
            k.op("LDG.E", [4], [10], base=buf(0) + ((s * bs + i) * n + s * bs) * 4, stride=4, mask=0xFFFF)
            k.op("STS", [], [4], base=i * 64, stride=4, mask=0xFFFF)
        k.op("BAR.SYNC")
        for i in range(bs - 1):
            act = (0xFFFF << (i + 1)) & 0xFFFF
            for j in range(max(1, i // 2)):
                k.op("LDS", [5], [2], base=i * 64, stride=4, mask=act)
                k.op("LDS", [6], [2], base=j * 64, stride=4, mask=act)
                k.op("FFMA", [7], [5, 6, 7], mask=act)
            k.op("STS", [], [7], base=i * 64, stride=4, mask=act)
            k.op("BAR.SYNC")
        for i in range(bs):
            k.op("LDS", [4], [2], base=i * 64, stride=4, mask=0xFFFF)
            k.op("STG.E", [], [10, 4], base=buf(0) + ((s * bs + i) * n + s * bs) * 4, stride=4, mask=0xFFFF)
        _epilogue(k)
        out.append(k.build())
        rem = steps - s - 1
        if rem == 0:
            break
        # perimeter
        k = KernelBuilder("_Z13lud_perimeterPfii", (rem, 1, 1), (2 * bs, 1, 1), shmem=3 * bs * bs * 4, nregs=32,
                          kid=kid)
        kid += 1
        g = k.g
        _prologue(k, 3)
        for i in range(bs // 2):
            k.op("LDG.E", [4], [10], base=buf(0) + ((s * bs + i) * n + (s + 1 + g.cta) * bs) * 4, stride=4)
            k.op("STS", [], [4], base=i * 64, stride=4)
        k.op("BAR.SYNC")
        for i in range(bs):
            for j in range(i // 3 + 1):
                k.op("LDS", [5], [2], base=j * 64, stride=4)
                k.op("LDS", [6], [2], base=i * 64 + 1024, stride=4)
                k.op("FFMA", [7], [5, 6, 7])
            k.op("STS", [], [7], base=i * 64 + 2048, stride=4)
        k.op("BAR.SYNC")
        for i in range(bs // 2):
            k.op("LDS", [4], [2], base=i * 64 + 2048, stride=4)
            k.op("STG.E", [], [10, 4], base=buf(0) + ((s * bs + i) * n + (s + 1 + g.cta) * bs) * 4, stride=4)
        _epilogue(k)
        out.append(k.build())
        # internal
        k = KernelBuilder("_Z12lud_internalPfii", (rem, rem, 1), (bs, bs, 1), shmem=2 * bs * bs * 4, nregs=20,
                          kid=kid)
        kid += 1
        g = k.g
        r0 = (s + 1 + g.cy) * bs + g.warp * 2
        c0 = (s + 1 + g.cx) * bs
        _prologue(k, 3)
        k.op("LDG.E", [4], [10], base=buf(0) + (r0 * n + s * bs) * 4, stride=4)
        k.op("LDG.E", [5], [11], base=buf(0) + ((s * bs + g.warp * 2) * n + c0) * 4, stride=4)
        k.op("STS", [], [4], base=g.warp * 128, stride=4)
        k.op("STS", [], [5], base=1024 + g.warp * 128, stride=4)
        k.op("BAR.SYNC")
        for i in range(bs):
            k.op("LDS", [6], [2], base=g.warp * 128 + (i % 2) * 64, stride=0)
            k.op("LDS", [7], [2], base=1024 + i * 64, stride=4)
            k.op("FFMA", [8], [6, 7, 8])
        k.op("LDG.E", [9], [12], base=buf(0) + (r0 * n + c0) * 4, stride=4)
        k.op("FADD", [9], [9, 8])
        k.op("STG.E", [], [12, 9], base=buf(0) + (r0 * n + c0) * 4, stride=4)
        _epilogue(k)
        out.append(k.build())
    return out


# ----------------------------------------------------------------------------
def nw(n: int = 128, penalty: int = 10, kid0: int = 1) -> List[KernelArrays]:
    """needle_cuda_shared_1 / _2: anti-diagonal wavefronts of 16x16 tiles."""
    bs = 16
    nb = n // bs
    out = []
    kid = kid0

    def tile_kernel(name, nblk, which):
        nonlocal kid
        k = KernelBuilder(name, (nblk, 1, 1), (bs, 1, 1), shmem=(bs + 1) * (bs + 1) * 4 + bs * bs * 4, nregs=30,
                          kid=kid)
        kid += 1
        g = k.g
        base = buf(0) + (g.cta * bs * (n + 1) + which) * 4
        _prologue(k, 3)
        k.op("LDG.E", [4], [10], base=base, stride=4, mask=0xFFFF)
        k.op("STS", [], [4], base=0, stride=4, mask=0xFFFF)
        for i in range(bs):
            k.op("LDG.E", [5], [11], base=base + (i + 1) * (n + 1) * 4, stride=4, mask=0xFFFF)
            k.op("STS", [], [5], base=(bs + 1) * 4 * (i + 1), stride=4, mask=0xFFFF)
        k.op("BAR.SYNC")
        for d in range(2 * bs - 1):
            act = 0
            for t in range(bs):
                if 0 <= d - t < bs:
                    act |= 1 << t
            k.op("LDS", [6], [2], base=d * 4, stride=(bs + 1) * 4 - 4, mask=act)
            k.op("LDS", [7], [2], base=d * 4 + 4, stride=(bs + 1) * 4 - 4, mask=act)
            k.op("LDS", [8], [2], base=d * 4 + (bs + 1) * 4, stride=(bs + 1) * 4 - 4, mask=act)
            k.op("IADD3", [9], [6, 7], mask=act)
            k.op("IMNMX", [9], [9, 8], mask=act)
            k.op("IMNMX", [9], [9, 6], mask=act)
            k.op("STS", [], [9], base=d * 4 + (bs + 2) * 4, stride=(bs + 1) * 4 - 4, mask=act)
            k.op("BAR.SYNC")
        for i in range(bs):
            k.op("LDS", [5], [2], base=(bs + 1) * 4 * (i + 1), stride=4, mask=0xFFFF)
            k.op("STG.E", [], [12, 5], base=base + (i + 1) * (n + 1) * 4, stride=4, mask=0xFFFF)
        _epilogue(k)
        out.append(k.build())

    for i in range(1, nb + 1):
        tile_kernel("_Z20needle_cuda_shared_1PiS_iiii", i, 0)
    for i in range(nb - 1, 0, -1):
        tile_kernel("_Z20needle_cuda_shared_2PiS_iiii", i, bs)
    return out


# ----------------------------------------------------------------------------
def nn(n_records: int = 42764, kid0: int = 1) -> List[KernelArrays]:
    """euclid: one distance per record (sqrt), coalesced float2 loads."""
    block = 256
    grid = -(-n_records // block)
    k = KernelBuilder("_Z6euclidP7latLongPfiff", (grid, 1, 1), (block, 1, 1), nregs=12, kid=kid0)
    g = k.g
    tid = g.cta * block + g.tid0
    live = np.clip(n_records - tid, 0, 32)
    mask = np.where(live >= 32, np.uint64(0xFFFFFFFF), ((np.uint64(1) << live.astype(np.uint64)) - np.uint64(1)))
    _prologue(k, 3)
    k.op("ISETP", [20], [2])
    k.op("LDG.E.64", [4], [10], base=buf(0) + tid * 8, stride=8, mask=mask)
    k.op("FADD", [6], [4, 7], mask=mask)
    k.op("FADD", [8], [5, 9], mask=mask)
    k.op("FMUL", [6], [6, 6], mask=mask)
    k.op("FFMA", [6], [8, 8, 6], mask=mask)
    k.op("MUFU.SQRT", [6], [6], mask=mask)
    k.op("STG.E", [], [11, 6], base=buf(1) + tid * 4, stride=4, mask=mask)
    _epilogue(k)
    return [k.build()]


# ----------------------------------------------------------------------------
def pathfinder(cols: int = 1000, rows: int = 20, pyramid: int = 5, kid0: int = 1) -> List[KernelArrays]:
    """dynproc_kernel: 256-thread blocks, `pyramid` rows per launch."""
    block = 256
    small = block - 2 * pyramid
    grid = -(-cols // small)
    out = []
    for it in range(max(1, (rows - 1) // pyramid)):
        k = KernelBuilder("_Z14dynproc_kerneliPiS_S_iiii", (grid, 1, 1), (block, 1, 1), shmem=2 * block * 4,
                          nregs=22, kid=kid0 + it)
        g = k.g
        col = np.clip(g.cta * small - pyramid + g.tid0, 0, cols - 32)
        _prologue(k, 3)
        k.op("LDG.E", [4], [10], base=buf(0) + col * 4, stride=4)
        k.op("STS", [], [4], base=g.warp * 128, stride=4)
        k.op("BAR.SYNC")
        for r in range(pyramid):
            k.op("ISETP", [20], [2])
            k.op("LDS", [5], [2], base=g.warp * 128 - 4, stride=4)
            k.op("LDS", [6], [2], base=g.warp * 128, stride=4)
            k.op("LDS", [7], [2], base=g.warp * 128 + 4, stride=4)
            k.op("IMNMX", [8], [5, 6])
            k.op("IMNMX", [8], [8, 7])
            k.op("LDG.E", [9], [11], base=buf(1) + ((it * pyramid + r) * cols + col) * 4, stride=4)
            k.op("IADD3", [8], [8, 9])
            k.op("BAR.SYNC")
            k.op("STS", [], [8], base=1024 + g.warp * 128, stride=4)
            k.op("BAR.SYNC")
            k.op("LDS", [4], [2], base=1024 + g.warp * 128, stride=4)
            k.op("STS", [], [4], base=g.warp * 128, stride=4)
        k.op("STG.E", [], [12, 4], base=buf(2) + col * 4, stride=4)
        _epilogue(k)
        out.append(k.build())
    return out


# ----------------------------------------------------------------------------
def srad_v2(rows: int = 128, cols: int = 128, iters: int = 2, kid0: int = 1) -> List[KernelArrays]:
    """srad_cuda_1 (gradients, diffusion coefficient) + srad_cuda_2 (update)."""
    bs = 16
    grid = (cols // bs, rows // bs, 1)
    out = []
    kid = kid0
    for _ in range(iters):
        for kname, heavy in (("_Z11srad_cuda_1PfS_S_S_S_S_iif", True), ("_Z11srad_cuda_2PfS_S_S_S_S_iiff", False)):
            k = KernelBuilder(kname, grid, (bs, bs, 1), shmem=6 * bs * bs * 4, nregs=40, kid=kid)
            kid += 1
            g = k.g
            r = g.cy * bs + g.warp * 2
            addr = (r * cols + g.cx * bs) * 4
            _prologue(k, 4)
            for i in range(4 if heavy else 3):
                k.op("LDG.E", [4 + i], [10], base=buf(i) + addr, stride=4)
                k.op("STS", [], [4 + i], base=i * 1024 + g.warp * 128, stride=4)
            k.op("BAR.SYNC")
            for i in range(4):
                k.op("LDS", [8 + i], [2], base=i * 1024 + g.warp * 128 + 4 * ((i % 3) - 1), stride=4)
                k.op("FADD", [12 + i], [8 + i, 4])
            if heavy:
                k.op("FMUL", [16], [12, 12])
                k.op("FFMA", [16], [13, 13, 16])
                k.op("FFMA", [16], [14, 14, 16])
                k.op("FFMA", [16], [15, 15, 16])
                k.op("MUFU.RCP", [17], [4])
                k.op("FMUL", [16], [16, 17])
                k.op("FMUL", [18], [17, 17])
                k.op("FFMA", [18], [16, 18, 19])
                k.op("MUFU.RCP", [19], [18])
                k.op("FSETP", [22], [19])
                k.op("FSEL", [19], [19])
            else:
                for i in range(4):
                    k.op("FFMA", [16], [12 + i, 8 + i, 16])
                k.op("FFMA", [16], [16, 17, 4])
            k.op("STG.E", [], [11, 16], base=buf(4) + addr, stride=4)
            if heavy:
                k.op("STG.E", [], [11, 19], base=buf(5) + addr, stride=4)
            _epilogue(k)
            out.append(k.build())
    return out


# ----------------------------------------------------------------------------
def streamcluster(n_points: int = 1024, dim: int = 16, launches: int = 24, kid0: int = 1) -> List[KernelArrays]:
    """kernel_compute_cost: one launch per pgain() candidate."""
    block = 512
    grid = -(-n_points // block)
    out = []
    for it in range(launches):
        k = KernelBuilder("_Z19kernel_compute_costiilP5PointiiPfS1_PiPb", (grid, 1, 1), (block, 1, 1),
                          shmem=dim * 4, nregs=28, kid=kid0 + it)
        g = k.g
        tid = g.cta * block + g.tid0
        _prologue(k, 3)
        k.op("ISETP", [20], [2])
        k.op("LDG.E", [4], [10], base=buf(0) + ((it * 7) % n_points) * dim * 4, stride=0, mask=0xFFFF)
        k.op("STS", [], [4], base=0, stride=4, mask=0xFFFF)
        k.op("BAR.SYNC")
        for d in range(dim):
            k.op("LDG.E", [5], [11], base=buf(1) + (d * n_points + tid) * 4, stride=4)  # coord (transposed)
            k.op("LDS", [6], [2], base=d * 4, stride=0)
            k.op("FADD", [7], [5, 6])
            k.op("FFMA", [8], [7, 7, 8])
        k.op("LDG.E", [9], [12], base=buf(2) + tid * 4, stride=4)   # weight
        k.op("LDG.E", [13], [12], base=buf(3) + tid * 4, stride=4)  # cost
        k.op("FMUL", [8], [8, 9])
        k.op("FSETP", [21], [8, 13])
        k.op("STG.E", [], [12, 8], base=buf(4) + tid * 4, stride=4)
        k.op("LDG.E", [14], [12], base=buf(5) + tid * 4, stride=4)  # assign
        k.op("FADD", [15], [13, 8])
        k.op("STG.E", [], [12, 15], base=buf(6) + (tid % 64) * 4, stride=4)
        _epilogue(k)
        out.append(k.build())
    return out


# ----------------------------------------------------------------------------
# v2 (round 5): heartwall with the measured gfx950 instruction mix (~10 vector
# ALU per global load, 7.05 M thread instructions: the reference's "7 M",
# profiles/heartwall_parity.md); v1 used heartwall(51, scale=2.0) (6.53 M, IPC
# 451 against the reference's 883).  Cached traces are keyed by the version.
SUITE_VERSION = 2
SUITE: Dict[str, Tuple[str, Callable[..., List[KernelArrays]]]] = {
    # name: (argument folder as in define-all-apps.yml, generator)
    "backprop-rodinia-2.0-ft": ("4096___data_result_4096_txt", lambda: backprop(4096)),
    "bfs-rodinia-2.0-ft": ("__data_graph4096_txt___data_graph4096_result_txt", lambda: bfs(4096)),
    "hotspot-rodinia-2.0-ft": ("30_6_40___data_result_30_6_40_txt", lambda: hotspot(256, 2, 6)),
    "heartwall-rodinia-2.0-ft": ("__data_test_avi_1___data_result_1_txt",
                                 lambda: heartwall(51, scale=1.0, alu_per_iter=14)),
    "lud-rodinia-2.0-ft": ("_v__b__i___data_64_dat", lambda: lud(64)),
    "nw-rodinia-2.0-ft": ("128_10___data_result_128_10_txt", lambda: nw(128, 10)),
    "nn-rodinia-2.0-ft": ("__data_filelist_4_3_30_90___data_filelist_4_3_30_90_result_txt", lambda: nn(42764)),
    "pathfinder-rodinia-2.0-ft": ("1000_20_5___data_result_1000_20_5_txt", lambda: pathfinder(1000, 20, 5)),
    "srad_v2-rodinia-2.0-ft": ("__data_matrix128x128_txt_0_127_0_127__5_2___data_result_matrix128x128_1_150_1_100__5_2_txt",
                               lambda: srad_v2(128, 128, 2)),
    "streamcluster-rodinia-2.0-ft": ("3_6_16_1024_1024_100_none_output_txt_1___data_result_3_6_16_1024_1024_100_none_1_txt",
                                     lambda: streamcluster(1024, 16, 24)),
}


def _memcpys(kernels: List[KernelArrays]) -> List[str]:
    # H2D copies of the input buffers touched by the first kernel (bounded)
    lines = []
    if not kernels:
        return lines
    mems = kernels[0].mems
    if len(mems):
        bufs = sorted(set(int(b) // BUF * BUF for b in mems["base"] if b))
        for b in bufs[:4]:
            lines.append(f"MemcpyHtoD,0x{b:016x},{1 << 20}")
    return lines


def write_app(out_dir: str, kernels: List[KernelArrays], text: bool = False, memcpy: bool = True) -> str:
    """Write one application's traces; returns the kernelslist.g path."""
    os.makedirs(out_dir, exist_ok=True)
    cmds = _memcpys(kernels) if memcpy else []
    for i, k in enumerate(kernels, 1):
        k.header["id"] = i
        if text:
            fn = f"kernel-{i}.traceg"
            write_kernel_text(os.path.join(out_dir, fn), k)
        else:
            fn = f"kernel-{i}.asimk"
            write_kernel_binary(os.path.join(out_dir, fn), k)
        cmds.append(fn)
    return write_kernelslist(out_dir, cmds)


def generate_suite(root: str, apps=None, text: bool = False) -> Dict[str, str]:
    """Generate the Rodinia-2.0-ft-shaped suite under ``root``.

    Layout matches the reference's hw_run/traces tree:
    ``<root>/<app>/<args>/traces/kernelslist.g``.  Returns {app: kernelslist}.
    """
    out = {}
    for app, (args, gen) in SUITE.items():
        if apps and app not in apps:
            continue
        d = os.path.join(root, app, args, "traces")
        out[app] = write_app(d, gen(), text=text)
    return out


def suite_stats(root: str) -> Dict[str, Dict[str, int]]:
    from .format import read_kernel_binary
    res = {}
    for app, (args, _) in SUITE.items():
        d = os.path.join(root, app, args, "traces")
        if not os.path.isdir(d):
            continue
        ti = wi = nk = 0
        for fn in sorted(os.listdir(d)):
            if fn.endswith(".asimk"):
                k = read_kernel_binary(os.path.join(d, fn))
                ti += k.thread_insts
                wi += len(k.insts)
                nk += 1
        res[app] = dict(kernels=nk, warp_insts=wi, thread_insts=ti)
    return res


# ----------------------------------------------------------------------------
def test_kernel(kid: int = 1) -> KernelArrays:
    """examples/all-reduce test_kernel<<<1,256>>>: ptr[threadIdx.x] = 7."""
    k = KernelBuilder("_Z11test_kernelPi", (1, 1, 1), (256, 1, 1), nregs=8, kid=kid)
    g = k.g
    k.op("S2R", [0])
    k.op("MOV", [1])
    k.op("IMAD.WIDE", [2], [0, 1])
    k.op("STG.E", [], [2, 1], base=buf(7) + g.tid0 * 4, stride=4)
    k.op("EXIT")
    return k.build()


def write_allreduce_example(out_dir: str, nranks: int = 1, count: int = 32 * 1024 * 1024) -> str:
    """Trace of examples/all-reduce (main.cu): memcpys, two test kernels around
    an ncclAllReduce of `count` floats, with the collective's arguments
    recorded (the reference's tracer drops them)."""
    os.makedirs(out_dir, exist_ok=True)
    for i in (1, 2):
        write_kernel_binary(os.path.join(out_dir, f"kernel-{i}.asimk"), test_kernel(i))
    cmds = [
        f"MemcpyHtoD,0x{buf(8):016x},{count * 4}",
        f"ncclCommInitAll,nranks={nranks}",
        "kernel-1.asimk",
        "ncclGroupStart",
        f"ncclAllReduce,count={count},dtype=ncclFloat,op=ncclSum,nranks={nranks}",
        "ncclGroupEnd",
        "kernel-2.asimk",
        "ncclCommDestroy",
    ]
    return write_kernelslist(out_dir, cmds)
