"""Vectorised warp-program builder for synthetic kernel traces.

A kernel is described as ONE straight-line warp program (loops unrolled by
the caller) whose memory operands are functions of (cta, warp, iteration):
every column of the program is emitted for all warps at once with numpy, so
multi-million-instruction kernels are generated in well under a second.
Per-warp differences (tail warps, early exit, divergence) are expressed with
a per-warp ``present`` flag and per-warp active masks.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Union

import numpy as np

from .format import NO_MEM, SASS, TINST, TMEM, WSTREAM, KernelArrays, op_info

ArrayLike = Union[int, np.ndarray]


class WarpGrid:
    """Index helpers for all warps of a kernel (row-major CTA order)."""

    def __init__(self, grid, block, warp_size=32):
        self.grid = tuple(int(x) for x in grid) + (1,) * (3 - len(grid))
        self.block = tuple(int(x) for x in block) + (1,) * (3 - len(block))
        self.warp_size = warp_size
        self.threads = int(np.prod(self.block))
        self.wpc = -(-self.threads // warp_size)
        self.ncta = int(np.prod(self.grid))
        self.nwarps = self.ncta * self.wpc
        w = np.arange(self.nwarps, dtype=np.int64)
        self.cta = w // self.wpc                      # linear CTA id
        self.warp = w % self.wpc                      # warp in CTA
        self.cx = self.cta % self.grid[0]
        self.cy = (self.cta // self.grid[0]) % self.grid[1]
        self.cz = self.cta // (self.grid[0] * self.grid[1])
        self.tid0 = self.warp * warp_size             # first thread id of the warp in its CTA
        self.gtid0 = self.cta * self.threads + self.tid0
        # active mask of full / tail warps
        live = np.minimum(warp_size, self.threads - self.tid0)
        full = (1 << warp_size) - 1
        self.full_mask = np.where(live >= warp_size, full, (1 << np.maximum(live, 0)) - 1).astype(np.uint64)


class KernelBuilder:
    def __init__(self, name: str, grid, block, shmem: int = 0, nregs: int = 32, binary_version: int = 70,
                 warp_size: int = 32, kid: int = 1, seed: int = 0):
        self.g = WarpGrid(grid, block, warp_size)
        self.header = dict(name=name, id=kid, grid=self.g.grid, block=self.g.block, shmem=shmem, nregs=nregs,
                           binary_version=binary_version, warp_size=warp_size, trace_version=4,
                           shmem_base=0x00007F0000000000, local_base=0x00007F1000000000)
        self.cols: List[Dict] = []
        self.rng = np.random.default_rng(seed)
        self.pc = 0
        self.opnames: List[str] = ["<none>"]
        self.opids: Dict[str, int] = {}

    # ---- emission ----------------------------------------------------------
    def _opid(self, m: str) -> int:
        if m not in self.opids:
            self.opids[m] = len(self.opnames)
            self.opnames.append(m)
        return self.opids[m]

    def op(self, mnemonic: str, dst: Sequence[int] = (), src: Sequence[int] = (), *,
           base: Optional[ArrayLike] = None, stride: Optional[int] = None,
           addrs: Optional[np.ndarray] = None, mask: Optional[ArrayLike] = None,
           present: Optional[np.ndarray] = None) -> None:
        """Emit one instruction for every warp.

        Memory ops take either ``base`` (per-warp array or scalar) + ``stride``
        (bytes between consecutive active lanes) or ``addrs`` [nwarps, lanes].
        """
        cls, space, flags, width = op_info(mnemonic)
        n = self.g.nwarps
        col = dict(op=self._opid(mnemonic), cls=cls, space=space, flags=flags, width=width,
                   dst=tuple(dst)[:2], src=tuple(src)[:5], pc=self.pc,
                   mask=self.g.full_mask if mask is None else np.broadcast_to(
                       np.asarray(mask, np.uint64), (n,)) & self.g.full_mask,
                   present=np.ones(n, bool) if present is None else np.asarray(present, bool),
                   base=None, stride=None, addrs=None)
        if flags & 4:  # memory
            if addrs is not None:
                col["addrs"] = np.asarray(addrs, np.uint64)
            else:
                col["base"] = np.broadcast_to(np.asarray(base, np.int64), (n,)).astype(np.uint64)
                col["stride"] = int(width if stride is None else stride)
        self.cols.append(col)
        self.pc += 16

    def alu(self, mnemonic: str, n: int = 1, regs=(4, 5, 6), present=None, mask=None) -> None:
        """n dependent-ish ALU ops cycling through a small register window."""
        for i in range(n):
            d = regs[i % len(regs)]
            s1 = regs[(i + 1) % len(regs)]
            s2 = regs[(i + 2) % len(regs)]
            self.op(mnemonic, [d], [s1, s2], present=present, mask=mask)

    # ---- assembly ------------------------------------------------------------
    def build(self) -> KernelArrays:
        n = self.g.nwarps
        L = len(self.cols)
        ins = np.zeros((n, L), TINST)
        present = np.zeros((n, L), bool)
        # memory bookkeeping: per (warp, col) mem row, filled after compaction
        for j, c in enumerate(self.cols):
            col = ins[:, j]
            col["pc"] = c["pc"]
            col["opcode"] = c["op"]
            col["cls"] = c["cls"]
            col["space"] = c["space"]
            col["flags"] = c["flags"]
            col["width"] = c["width"]
            col["mask"] = c["mask"]
            for k, r in enumerate(c["dst"]):
                col["dst"][:, k] = r + 1
            for k, r in enumerate(c["src"]):
                col["src"][:, k] = r + 1
            col["mem"] = NO_MEM
            present[:, j] = c["present"] & (c["mask"] != 0) | (c["present"] & (c["cls"] in (9, 11)))
        # memory rows in the final (warp-major) instruction order
        mem_rows = []
        addr_chunks = []
        addr_off = 0
        mem_index = np.full((n, L), NO_MEM, np.uint64)
        nmem = 0
        for j, c in enumerate(self.cols):
            if not (c["flags"] & 4):
                continue
            sel = present[:, j]
            cnt = int(sel.sum())
            if cnt == 0:
                continue
            rows = np.zeros(cnt, TMEM)
            if c["addrs"] is None:
                rows["base"] = c["base"][sel]
                rows["stride"] = c["stride"]
                rows["list"] = NO_MEM
            else:
                a = c["addrs"][sel]
                m = c["mask"][sel]
                lanes = a.shape[1]
                bits = ((m[:, None] >> np.arange(lanes, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
                nact = bits.sum(1)
                starts = addr_off + np.concatenate([[0], np.cumsum(nact)[:-1]])
                rows["base"] = np.where(nact > 0, a[np.arange(cnt), np.argmax(bits, 1)], 0)
                rows["stride"] = 0
                rows["list"] = starts.astype(np.uint32)
                addr_chunks.append(a[bits])
                addr_off += int(nact.sum())
            mem_rows.append(rows)
            mem_index[sel, j] = np.arange(nmem, nmem + cnt, dtype=np.uint64)
            nmem += cnt
        ins["mem"] = np.where(mem_index == NO_MEM, NO_MEM, mem_index).astype(np.uint32)
        # compaction: per-warp contiguous streams
        counts = present.sum(1)
        flat = ins[present]
        begins = np.concatenate([[0], np.cumsum(counts)[:-1]])
        streams = np.zeros(n, WSTREAM)
        streams["begin"] = begins
        streams["count"] = counts
        mems = np.concatenate(mem_rows) if mem_rows else np.zeros(0, TMEM)
        addrs = np.concatenate(addr_chunks).astype(np.uint64) if addr_chunks else np.zeros(0, np.uint64)
        return KernelArrays(self.header, flat, mems, addrs, streams, self.opnames)
