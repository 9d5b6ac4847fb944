"""gfx950 assembly instrumentation: the ISA-level half of the automatic tracer.

Reference: the NVBit tracer instruments every SASS instruction of an
unmodified binary at load time (util/tracer_nvbit/tracer_tool/
tracer_tool.cu:130-275 ``instrument_function_if_needed``) and its injected
device functions push the active mask and 32 lane addresses per instruction
into a channel (inject_funcs.cu:20-81).  CDNA4 has no binary-instrumentation
framework in this stack, so the same information is captured by rewriting the
compiler's own gfx950 assembly of the unmodified HIP source before it is
assembled (``hipcc -S --cuda-device-only``):

* the kernel code is cut into *segments* -- maximal instruction runs with one
  entry and a constant EXEC mask (a new segment starts at every label, after
  every branch and after every instruction that writes EXEC);
* a probe at the head of each segment appends a 16-byte record
  ``{segment id, 0, exec}`` to the wave's trace stream;
* a probe before each vector-memory / LDS instruction appends
  ``{0x80000000 | memory-op id, 0, exec}`` plus 64 per-lane 8-byte addresses
  computed from the instruction's own operands (global/flat/scratch/buffer/
  ds addressing modes);
* records go to 8 KB chunks; a wave claims a chunk with one atomic (a
  ticket) and tags it ``{0xC0000000 | chunk seq, wg x, wg y, wg z}`` +
  ``{packed thread id of the first lane, 0, 0, slot generation}``, so the host
  regroups chunks by wave without any ordering between waves;
* streaming (the default, ``ctl.mask != 0``): the chunks form a ring of
  ``mask + 1`` slots in coherent host memory.  Ticket ``t`` owns slot
  ``t & mask`` once the host has drained that slot's previous occupant
  (the slot's generation word reads ``t >> shift``; the wave polls it with
  system-scope loads, ``s_sleep`` between polls, and after ``SPIN_LIMIT``
  polls -- ``ctl.spin_limit``, set by the host -- gives up and stops
  recording rather than hang; the host then refuses to write that kernel's
  trace and fails the run: a capture is lossless or it is an error).  A wave leaving a
  full chunk writes a close marker into the chunk's last unit after its
  records have drained (``s_waitcnt vmcnt(0)``); the host's drain thread
  copies closed chunks out during the kernel and frees their slots, so no
  buffer bounds the trace of one kernel (reference: the NVBit channel,
  util/tracer_nvbit/nvbit_release/core/utils/channel.hpp:56-116,161-253,
  whose device side waits for the host to flush a full buffer).  Every probe
  store is system scope (``sc0 sc1``: written through the XCD L2);
* device-buffer mode (``mask == 0``): tickets index one device buffer of
  ``n_chunks`` chunks; a ticket past its end stops the wave's recording.

Probes use only registers above the kernel's own allocation (16 SGPRs, 8
VGPRs; the descriptor's counts are raised), save and restore SCC and EXEC,
never touch VCC or M0, and only *add* vector-memory operations, so every
``s_waitcnt`` of the original code stays correct (it can only wait longer).
The workgroup-id y/z system SGPRs are enabled so a wave knows its CTA; a
workgroup-info SGPR displaced by that is moved back at entry.

The static side -- every segment's instructions with their real byte offsets
(from disassembling the uninstrumented code object), register operands and
memory widths -- goes to a ``.asimisa`` map that the host runtime
(csrc/tracer/isa_runtime.cc) uses to expand the record stream into
``kernel-N.traceg`` files.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

CHUNK_UNITS = 512           # 16-byte units per chunk (8 KB; recorded in the map header)
TAG_MEM = 0x80000000
TAG_CHUNK = 0xC0000000
TAG_CLOSE = 0xE0000000      # last unit of a chunk a wave has left (streaming)
SPIN_LIMIT = 1 << 18        # generation polls before a wave stops recording
ST = "sc0 sc1"              # probe stores: system scope (the host reads them)
N_PROBE_SGPR = 16
N_PROBE_VGPR = 8
MAX_SGPR = 102
MAX_ARCH_VGPR = 256

_LABEL = re.compile(r"^([.\w$]+):")
_REG = re.compile(r"^(v|s|a)(\d+)$|^(v|s|a)\[(\d+):(\d+)\]$")


class RewriteError(RuntimeError):
    pass


@dataclass
class Inst:
    text: str                 # original line (no comment)
    mnem: str
    ops: List[str]            # comma-separated operands (modifiers stripped)
    mods: List[str]           # trailing modifiers (offset:N, glc, offen ...)
    pc: int = 0               # byte offset from the kernel entry (filled from the disassembly)
    mem_id: int = -1
    seg: int = 0


@dataclass
class Kernel:
    name: str
    start: int                # line index of the kernel label
    end: int                  # line index of .Lfunc_end
    insts: List[Inst] = field(default_factory=list)
    segments: List[List[int]] = field(default_factory=list)   # seg id-1 -> inst indices
    n_mem: int = 0


def parse_reg(tok: str) -> Optional[Tuple[str, int, int]]:
    """'v[4:5]' -> ('v', 4, 2); 's3' -> ('s', 3, 1); anything else None."""
    t = tok.strip()
    m = _REG.match(t)
    if not m:
        return None
    if m.group(1):
        return m.group(1), int(m.group(2)), 1
    lo, hi = int(m.group(4)), int(m.group(5))
    return m.group(3), lo, hi - lo + 1


def split_inst(line: str) -> Optional[Inst]:
    code = line.split(";", 1)[0].strip()
    if not code or code.startswith(".") or _LABEL.match(code):
        return None
    parts = code.split(None, 1)
    mnem = parts[0]
    rest = parts[1] if len(parts) > 1 else ""
    ops = [o.strip() for o in rest.split(",")] if rest else []
    mods: List[str] = []
    if ops:
        last = ops[-1].split()
        ops[-1] = last[0] if last else ""
        mods = last[1:]
        if ops[-1] == "":
            ops.pop()
    return Inst(code, mnem, ops, mods)


def mem_width(m: str) -> int:
    for k, w in (("dwordx4", 16), ("b128", 16), ("dwordx3", 12), ("b96", 12), ("dwordx2", 8), ("b64", 8),
                 ("x2", 8), ("short", 2), ("b16", 2), ("u16", 2), ("i16", 2), ("byte", 1), ("b8", 1), ("u8", 1),
                 ("i8", 1)):
        if k in m:
            return w
    return 4


def is_vector_mem(m: str) -> bool:
    if m.startswith(("global_", "flat_", "scratch_", "buffer_")):
        return not m.startswith(("buffer_wbl2", "buffer_inv", "buffer_wbinv", "buffer_gl"))
    if m.startswith("ds_"):
        return not m.startswith(("ds_append", "ds_consume", "ds_gws", "ds_nop", "ds_swizzle"))
    return False


def is_store(m: str) -> bool:
    return m.startswith(("global_store", "flat_store", "scratch_store", "buffer_store", "ds_write", "ds_store"))


def is_branch(m: str) -> bool:
    return m.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc", "s_call"))


def writes_exec(ins: Inst) -> bool:
    m = ins.mnem
    if "saveexec" in m or m.startswith("v_cmpx"):
        return True
    if m.startswith("s_") and ins.ops and ins.ops[0] in ("exec", "exec_lo", "exec_hi"):
        return True
    return False


def _no_dst(m: str) -> bool:
    return (is_store(m) or is_branch(m) or m.startswith(("s_cmp", "s_bitcmp", "s_waitcnt", "s_barrier", "s_endpgm",
                                                          "s_nop", "s_sleep", "s_setprio", "s_sched", "s_dcache",
                                                          "s_icache", "s_sendmsg", "s_trap", "s_ttrace"))
            or (m.startswith("ds_") and not any(k in m for k in ("read", "load", "rtn", "permute")))
            or (m.startswith(("buffer_atomic", "global_atomic", "flat_atomic"))))


def reg_operands(ins: Inst) -> Tuple[List[str], List[str]]:
    """(destination, source) register names for the trace, first two
    registers of a destination tuple and the first of each source tuple."""
    regs = []
    for o in ins.ops:
        r = parse_reg(o)
        regs.append(r)
    dst: List[str] = []
    src: List[str] = []
    start = 0
    m = ins.mnem
    atomic_rtn = m.startswith(("global_atomic", "flat_atomic", "buffer_atomic")) and any(
        x in ins.mods for x in ("glc", "sc0"))
    if (not _no_dst(m)) or atomic_rtn:
        if regs and regs[0] is not None:
            k, lo, n = regs[0]
            dst = [f"{k}{lo + i}" for i in range(min(n, 2))]
        start = 1
    for r in regs[start:]:
        if r is not None:
            src.append(f"{r[0]}{r[1]}")
    return dst, src


# ----------------------------------------------------------------------------- parsing
def parse_kernels(lines: Sequence[str]) -> Dict[str, Kernel]:
    names = set()
    for ln in lines:
        s = ln.strip()
        if s.startswith(".amdhsa_kernel "):
            names.add(s.split()[1])
    return parse_bodies(lines, names)


_FUNC_TYPE = re.compile(r"^\s*\.type\s+([.\w$]+)\s*,\s*@function")


def function_names(lines: Sequence[str]) -> set:
    """Every symbol declared ``.type name,@function`` (kernels included)."""
    out = set()
    for ln in lines:
        m = _FUNC_TYPE.match(ln)
        if m:
            out.add(m.group(1))
    return out


def parse_bodies(lines: Sequence[str], names) -> Dict[str, Kernel]:
    """The instruction bodies of the named functions (label to .Lfunc_end)."""
    kernels: Dict[str, Kernel] = {}
    i = 0
    while i < len(lines):
        m = _LABEL.match(lines[i])
        if m and m.group(1) in names:
            name = m.group(1)
            j = i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                if lines[j].lstrip().startswith(".section") and ".rodata" in lines[j]:
                    break
                j += 1
            k = Kernel(name, i, j)
            for ln in lines[i + 1:j]:
                ins = split_inst(ln)
                if ins is not None:
                    k.insts.append(ins)
            kernels[name] = k
            i = j
        i += 1
    return kernels


def segment(k: Kernel, lines: Sequence[str], seg_base: int = 0, mem_base: int = 0) -> List[Tuple[int, str]]:
    """Assign segments and memory ids; return the kernel body as a list of
    (kind, text) items: 'L' label line, 'I' instruction index, 'X' other.
    Device functions number theirs from ``seg_base`` / ``mem_base`` (ids
    shared by every kernel that may call them)."""
    body: List[Tuple[int, str]] = []
    idx = 0
    for ln in lines[k.start + 1:k.end]:
        code = ln.split(";", 1)[0].strip()
        if _LABEL.match(code):
            body.append((-1, ln))
        elif split_inst(ln) is not None:
            body.append((idx, ln))
            idx += 1
        else:
            body.append((-2, ln))
    seg = 0
    new = True
    for kind, _ in body:
        if kind == -1:
            new = True
            continue
        if kind < 0:
            continue
        ins = k.insts[kind]
        if new:
            seg += 1
            k.segments.append([])
            new = False
        ins.seg = seg_base + seg
        k.segments[seg - 1].append(kind)
        if is_vector_mem(ins.mnem):
            ins.mem_id = mem_base + k.n_mem
            k.n_mem += 1
        if is_branch(ins.mnem) or writes_exec(ins) or ins.mnem == "s_endpgm":
            new = True
    return body


# ----------------------------------------------------------------------------- probes
class Probe:
    def __init__(self, S: int, V: int, tag: str = "0"):
        self.S, self.V = S, V
        self.tag = tag            # makes the probe labels unique per kernel
        self.ctl = f"s[{S}:{S + 1}]"
        self.buf = f"s[{S + 2}:{S + 3}]"
        self.cur = f"s{S + 4}"
        self.end = f"s{S + 5}"
        self.tx = f"s[{S + 6}:{S + 7}]"
        self.tx_lo, self.tx_hi = f"s{S + 6}", f"s{S + 7}"
        self.scc = f"s{S + 8}"
        self.t = f"s{S + 9}"
        self.wg = [f"s{S + 10}", f"s{S + 11}", f"s{S + 12}"]
        self.ptid = f"s{S + 13}"
        self.seq = f"s{S + 14}"
        self.t2 = f"s{S + 15}"
        self.va = f"v[{V}:{V + 1}]"
        self.va_lo, self.va_hi = f"v{V}", f"v{V + 1}"
        self.hdr = f"v[{V + 2}:{V + 5}]"
        self.h = [f"v{V + 2}", f"v{V + 3}", f"v{V + 4}", f"v{V + 5}"]
        self.off = f"v{V + 6}"

    # -- pieces
    def _store_unit(self, tag: str, w1: str = "0", exec_words: bool = True, unit_off: int = 0) -> List[str]:
        """one lane writes {tag, w1, exec lo, exec hi} at unit cur+unit_off"""
        h = self.h
        out = [f"s_mov_b64 {self.tx}, exec",
               "s_mov_b64 exec, 1",
               f"v_mov_b32_e32 {h[0]}, {tag}",
               f"v_mov_b32_e32 {h[1]}, {w1}",
               f"v_mov_b32_e32 {h[2]}, {self.tx_lo}" if exec_words else f"v_mov_b32_e32 {h[2]}, 0",
               f"v_mov_b32_e32 {h[3]}, {self.tx_hi}" if exec_words else f"v_mov_b32_e32 {h[3]}, 0",
               f"s_lshl_b32 {self.t}, {self.cur}, 4"]
        if unit_off:
            out.append(f"s_add_u32 {self.t}, {self.t}, {unit_off * 16}")
        out += [f"v_mov_b32_e32 {self.off}, {self.t}",
                f"global_store_dwordx4 {self.off}, {self.hdr}, {self.buf} {ST}",
                f"s_mov_b64 exec, {self.tx}"]
        return out

    def entry(self, wg_sgprs: Sequence[int], info_move: Optional[Tuple[int, int]]) -> List[str]:
        out = []
        for i, r in enumerate(wg_sgprs):
            out.append(f"s_mov_b32 {self.wg[i]}, s{r}")
        if info_move:
            out.append(f"s_mov_b32 s{info_move[0]}, s{info_move[1]}")
        out += [f"v_readfirstlane_b32 {self.ptid}, v0",
                f"s_getpc_b64 {self.ctl}",
                f"s_add_u32 s{self.S}, s{self.S}, __asim_tctl@rel32@lo+4",
                f"s_addc_u32 s{self.S + 1}, s{self.S + 1}, __asim_tctl@rel32@hi+12",
                f"s_load_dwordx2 {self.buf}, {self.ctl}, 0x0",
                "s_waitcnt lgkmcnt(0)",
                f"s_mov_b32 {self.cur}, 0",
                f"s_mov_b32 {self.end}, 0",
                f"s_mov_b32 {self.seq}, 0"]
        return out

    def guarded(self, n: int, need: int, body: List[str], stubs: List[str]) -> List[str]:
        """SCC save, space check, chunk allocation (in line, jumped over when
        the chunk has room: every probe branch stays short however large the
        kernel), body, SCC restore."""
        out = [f"s_cselect_b32 {self.scc}, 1, 0",
               f"s_add_u32 {self.t}, {self.cur}, {need}",
               f"s_cmp_gt_u32 {self.t}, {self.end}",
               f"s_cbranch_scc0 .Lasim{self.tag}_ret_{n}"]
        out += self.alloc_stub(n)
        out += [f".Lasim{self.tag}_ret_{n}:"]
        out += body
        out += [f".Lasim{self.tag}_skip_{n}:",
                f"s_cmp_lg_u32 {self.scc}, 0"]
        return out

    def alloc_stub(self, n: int) -> List[str]:
        """claim the next chunk (a ticket); streaming mode closes the chunk
        being left and waits for the ticket's ring slot (module docstring)."""
        h = self.h
        L = f".Lasim{self.tag}"
        out = [f"s_bitcmp1_b32 {self.seq}, 29",          # gave up on the ring
               f"s_cbranch_scc1 {L}_full_{n}",
               f"s_load_dword {self.t2}, {self.ctl}, 0x10",  # ring mask (0: device buffer)
               "s_waitcnt lgkmcnt(0)",
               f"s_cmp_eq_u32 {self.t2}, 0",
               f"s_cbranch_scc1 {L}_take_{n}",
               f"s_cmp_eq_u32 {self.end}, 0",
               f"s_cbranch_scc1 {L}_take_{n}",
               # close the chunk being left: its records first, then the marker
               "s_waitcnt vmcnt(0)",
               f"s_mov_b64 {self.tx}, exec",
               "s_mov_b64 exec, 1",
               f"v_mov_b32_e32 {h[0]}, {TAG_CLOSE:#x}",
               f"v_mov_b32_e32 {h[1]}, 0",
               f"v_mov_b32_e32 {h[2]}, 0",
               f"v_mov_b32_e32 {h[3]}, 0",
               f"s_lshl_b32 {self.t}, {self.end}, 4",
               f"v_mov_b32_e32 {self.off}, {self.t}",
               f"global_store_dwordx4 {self.off}, {self.hdr}, {self.buf} {ST}",
               f"s_mov_b64 exec, {self.tx}",
               f"{L}_take_{n}:",
               f"s_mov_b64 {self.tx}, exec",
               "s_mov_b64 exec, 1",
               f"v_mov_b32_e32 {h[0]}, 1",
               f"v_mov_b32_e32 {self.off}, 8",
               f"global_atomic_add {h[1]}, {self.off}, {h[0]}, {self.ctl} sc0",
               "s_waitcnt vmcnt(0)",
               f"v_readfirstlane_b32 {self.t}, {h[1]}",
               f"s_mov_b64 exec, {self.tx}",
               "s_nop 4",
               f"s_cmp_eq_u32 {self.t2}, 0",
               f"s_cbranch_scc1 {L}_dev_{n}",
               # ring: slot = ticket & mask, generation = ticket >> shift
               f"s_and_b32 {self.end}, {self.t}, {self.t2}",
               f"s_load_dword {self.t2}, {self.ctl}, 0x14",
               "s_waitcnt lgkmcnt(0)",
               f"s_lshr_b32 {self.t2}, {self.t}, {self.t2}",
               f"s_mul_i32 {self.cur}, {self.end}, {CHUNK_UNITS}",
               # polls before giving up: the control block's limit (the host
               # fails the run if any wave gave up), SPIN_LIMIT when unset
               f"s_load_dword {self.end}, {self.ctl}, 0x18",
               "s_waitcnt lgkmcnt(0)",
               f"s_cmp_eq_u32 {self.end}, 0",
               f"s_cselect_b32 {self.end}, {SPIN_LIMIT:#x}, {self.end}",
               f"s_mov_b64 {self.tx}, exec",
               "s_mov_b64 exec, 1",
               f"{L}_spin_{n}:",
               f"s_lshl_b32 {self.t}, {self.cur}, 4",
               f"s_add_u32 {self.t}, {self.t}, 28",           # unit 1, word 3
               f"v_mov_b32_e32 {self.off}, {self.t}",
               f"global_load_dword {h[1]}, {self.off}, {self.buf} sc0 sc1",
               "s_waitcnt vmcnt(0)",
               f"v_readfirstlane_b32 {self.t}, {h[1]}",
               f"s_cmp_eq_u32 {self.t}, {self.t2}",
               f"s_cbranch_scc1 {L}_got_{n}",
               f"s_sub_u32 {self.end}, {self.end}, 1",
               f"s_cmp_eq_u32 {self.end}, 0",
               f"s_cbranch_scc1 {L}_drop_{n}",
               "s_sleep 2",
               f"s_branch {L}_spin_{n}",
               f"{L}_drop_{n}:",
               f"s_mov_b64 exec, {self.tx}",
               f"s_bitset1_b32 {self.seq}, 29",
               f"s_branch {L}_full_{n}",
               f"{L}_got_{n}:",
               f"s_mov_b64 exec, {self.tx}",
               f"s_add_u32 {self.end}, {self.cur}, {CHUNK_UNITS - 1}",   # last unit: close marker
               f"s_branch {L}_hdr_{n}",
               f"{L}_dev_{n}:",
               f"s_load_dword {self.t2}, {self.ctl}, 0xc",
               "s_waitcnt lgkmcnt(0)",
               f"s_cmp_ge_u32 {self.t}, {self.t2}",
               f"s_cbranch_scc1 {L}_full_{n}",
               f"s_mul_i32 {self.cur}, {self.t}, {CHUNK_UNITS}",
               f"s_add_u32 {self.end}, {self.cur}, {CHUNK_UNITS}",
               f"{L}_hdr_{n}:"]
        # header unit 1: {ptid, 0, 0, generation (ring) | n_chunks}; unit 0:
        # {TAG_CHUNK|seq, wg x, wg y, wg z}, written last
        out += [f"s_mov_b64 {self.tx}, exec",
                "s_mov_b64 exec, 1",
                f"v_mov_b32_e32 {h[0]}, {self.ptid}",
                f"v_mov_b32_e32 {h[1]}, 0",
                f"v_mov_b32_e32 {h[2]}, 0",
                f"v_mov_b32_e32 {h[3]}, {self.t2}",
                f"s_lshl_b32 {self.t}, {self.cur}, 4",
                f"s_add_u32 {self.t}, {self.t}, 16",
                f"v_mov_b32_e32 {self.off}, {self.t}",
                f"global_store_dwordx4 {self.off}, {self.hdr}, {self.buf} {ST}",
                f"s_or_b32 {self.t2}, {self.seq}, {TAG_CHUNK:#x}",
                f"v_mov_b32_e32 {h[0]}, {self.t2}",
                f"v_mov_b32_e32 {h[1]}, {self.wg[0]}",
                f"v_mov_b32_e32 {h[2]}, {self.wg[1]}",
                f"v_mov_b32_e32 {h[3]}, {self.wg[2]}",
                f"s_sub_u32 {self.t}, {self.t}, 16",
                f"v_mov_b32_e32 {self.off}, {self.t}",
                f"global_store_dwordx4 {self.off}, {self.hdr}, {self.buf} {ST}",
                f"s_mov_b64 exec, {self.tx}",
                f"s_add_u32 {self.seq}, {self.seq}, 1",
                f"s_add_u32 {self.cur}, {self.cur}, 2",
                f"s_branch {L}_ret_{n}",
                f"{L}_full_{n}:",
                f"s_mov_b32 {self.cur}, 0",
                f"s_mov_b32 {self.end}, 0",
                f"s_branch {L}_skip_{n}"]
        return out

    def close_at_end(self, n: int) -> List[str]:
        """before s_endpgm (streaming): close the wave's last chunk so its
        slot can be drained while the kernel still runs"""
        h = self.h
        L = f".Lasim{self.tag}"
        return [f"s_load_dword {self.t2}, {self.ctl}, 0x10",
                "s_waitcnt lgkmcnt(0)",
                f"s_cmp_eq_u32 {self.t2}, 0",
                f"s_cbranch_scc1 {L}_endc_{n}",
                f"s_cmp_eq_u32 {self.end}, 0",
                f"s_cbranch_scc1 {L}_endc_{n}",
                "s_waitcnt vmcnt(0)",
                "s_mov_b64 exec, 1",
                f"v_mov_b32_e32 {h[0]}, {TAG_CLOSE:#x}",
                f"v_mov_b32_e32 {h[1]}, 0",
                f"v_mov_b32_e32 {h[2]}, 0",
                f"v_mov_b32_e32 {h[3]}, 0",
                f"s_lshl_b32 {self.t}, {self.end}, 4",
                f"v_mov_b32_e32 {self.off}, {self.t}",
                f"global_store_dwordx4 {self.off}, {self.hdr}, {self.buf} {ST}",
                f"{L}_endc_{n}:"]

    def segment(self, n: int, seg_id: int, stubs: List[str]) -> List[str]:
        body = self._store_unit(str(seg_id)) + [f"s_add_u32 {self.cur}, {self.cur}, 1"]
        return self.guarded(n, 1, body, stubs)

    # -- addresses
    def _add_sgpr_imm(self, val: int) -> List[str]:
        """64-bit v[va] += sext(val)"""
        if val == 0:
            return []
        hi = -1 if val < 0 else 0
        return [f"s_mov_b32 {self.t}, {val & 0xffffffff:#x}",
                f"v_add_co_u32_e64 {self.va_lo}, {self.tx}, {self.t}, {self.va_lo}",
                f"v_addc_co_u32_e64 {self.va_hi}, {self.tx}, {hi}, {self.va_hi}, {self.tx}"]

    def _add_sgpr(self, sreg: str) -> List[str]:
        return [f"v_add_co_u32_e64 {self.va_lo}, {self.tx}, {sreg}, {self.va_lo}",
                f"v_addc_co_u32_e64 {self.va_hi}, {self.tx}, 0, {self.va_hi}, {self.tx}"]

    def _add_vgpr32(self, vreg: str) -> List[str]:
        return [f"v_add_co_u32_e64 {self.va_lo}, {self.tx}, {vreg}, {self.va_lo}",
                f"v_addc_co_u32_e64 {self.va_hi}, {self.tx}, 0, {self.va_hi}, {self.tx}"]

    def address(self, ins: Inst) -> List[str]:
        m, ops = ins.mnem, ins.ops
        off = 0
        for md in ins.mods:
            if md.startswith("offset:"):
                off = int(md.split(":", 1)[1], 0)
            elif md.startswith("offset0:"):
                off = int(md.split(":", 1)[1], 0) * mem_width(m)
        va_lo, va_hi = self.va_lo, self.va_hi
        if m.startswith("ds_"):
            a = ops[1] if any(k in m for k in ("read", "load", "rtn", "permute")) else ops[0]
            r = parse_reg(a)
            if r is None:
                raise RewriteError(f"cannot parse LDS address of '{ins.text}'")
            return [f"v_add_u32_e32 {va_lo}, {off:#x}, v{r[1]}", f"v_mov_b32_e32 {va_hi}, 0"]
        if m.startswith(("global_", "flat_", "scratch_")):
            lds_dma = "_lds_" in m or m.endswith("_lds")
            if m.startswith("flat_"):
                saddr = "off"
                if is_store(m):
                    a = ops[0]
                elif "atomic" in m:
                    a = ops[1] if len(ops) == 3 else ops[0]
                else:
                    a = ops[1]
            else:
                saddr = ops[-1]
                if lds_dma:
                    a = ops[0]
                elif is_store(m):
                    a = ops[0]
                elif "atomic" in m:
                    a = ops[1] if len(ops) == 4 else ops[0]
                else:
                    a = ops[1]
            out: List[str] = []
            if m.startswith("scratch_"):
                # private (scratch) address: 32-bit offset within the wave's segment
                r = parse_reg(a)
                out.append(f"v_mov_b32_e32 {va_lo}, {'v%d' % r[1] if r else 0}")
                out.append(f"v_mov_b32_e32 {va_hi}, 0")
                if saddr != "off":
                    out.append(f"v_add_u32_e32 {va_lo}, {saddr}, {va_lo}")
                if off:
                    out.append(f"v_add_u32_e32 {va_lo}, {off & 0xffffffff:#x}, {va_lo}")
                return out
            r = parse_reg(a)
            if r is None:
                raise RewriteError(f"cannot parse address of '{ins.text}'")
            if saddr == "off":
                out += [f"v_mov_b32_e32 {va_lo}, v{r[1]}", f"v_mov_b32_e32 {va_hi}, v{r[1] + 1}"]
            else:
                sr = parse_reg(saddr)
                out += [f"v_mov_b32_e32 {va_lo}, v{r[1]}", f"v_mov_b32_e32 {va_hi}, 0"]
                out += self._add_sgpr(f"s{sr[1]}")
                out += [f"v_mov_b32_e32 {self.off}, s{sr[1] + 1}",
                        f"v_add_u32_e32 {va_hi}, {va_hi}, {self.off}"]
            return out + self._add_sgpr_imm(off)
        if m.startswith("buffer_"):
            # ops: vdata|vdst, vaddr|off, s[rsrc:rsrc+3], soffset
            if len(ops) < 4:
                raise RewriteError(f"cannot parse buffer operands of '{ins.text}'")
            va, rs, so = ops[1], parse_reg(ops[2]), ops[3]
            r0 = rs[1]
            out = [f"s_and_b32 {self.t2}, s{r0 + 1}, 0xffff",
                   f"v_mov_b32_e32 {va_lo}, s{r0}",
                   f"v_mov_b32_e32 {va_hi}, {self.t2}"]
            sor = parse_reg(so)
            if sor is not None:
                out += self._add_sgpr(f"s{sor[1]}")
            else:
                try:
                    out += self._add_sgpr_imm(int(so, 0))
                except ValueError:
                    pass
            vr = parse_reg(va)
            idxen, offen = "idxen" in ins.mods, "offen" in ins.mods
            if vr is not None and (idxen or offen):
                if idxen:
                    out += [f"s_bfe_u32 {self.t2}, s{r0 + 1}, 0xe0010",
                            f"v_mul_lo_u32 {self.off}, {self.t2}, v{vr[1]}"]
                    out += self._add_vgpr32(self.off)
                if offen:
                    out += self._add_vgpr32(f"v{vr[1] + (1 if idxen else 0)}")
            return out + self._add_sgpr_imm(off)
        raise RewriteError(f"unsupported memory instruction '{ins.text}'")

    def memory(self, n: int, ins: Inst, stubs: List[str]) -> List[str]:
        body = self.address(ins)
        body += [f"v_mbcnt_lo_u32_b32 {self.off}, -1, 0",
                 f"v_mbcnt_hi_u32_b32 {self.off}, -1, {self.off}",
                 f"v_lshlrev_b32_e32 {self.off}, 3, {self.off}",
                 f"s_lshl_b32 {self.t}, {self.cur}, 4",
                 f"s_add_u32 {self.t}, {self.t}, 16",
                 f"v_add_u32_e32 {self.off}, {self.t}, {self.off}",
                 f"global_store_dwordx2 {self.off}, {self.va}, {self.buf} {ST}"]
        body += self._store_unit(f"{TAG_MEM | ins.mem_id:#x}")
        body += [f"s_add_u32 {self.cur}, {self.cur}, 33"]
        return self.guarded(n, 33, body, stubs)


# ----------------------------------------------------------------------------- descriptor
_DIRECTIVE = re.compile(r"^(\s*)(\.amdhsa_[a-z0-9_]+)\s+(\S+)")


def _descriptor_block(lines: List[str], name: str) -> Tuple[int, int]:
    for i, ln in enumerate(lines):
        if ln.strip() == f".amdhsa_kernel {name}":
            for j in range(i + 1, len(lines)):
                if lines[j].strip() == ".end_amdhsa_kernel":
                    return i, j
    raise RewriteError(f"no kernel descriptor for {name}")


def _dget(lines, a, b, key, default=None):
    for i in range(a, b):
        m = _DIRECTIVE.match(lines[i])
        if m and m.group(2) == key:
            try:
                return int(m.group(3), 0), i
            except ValueError:
                raise RewriteError(f"{key} is an expression ({m.group(3)}); not supported")
    return default, -1


def _dset(lines, a, b, key, val) -> int:
    for i in range(a, b):
        m = _DIRECTIVE.match(lines[i])
        if m and m.group(2) == key:
            lines[i] = f"{m.group(1)}{key} {val}"
            return b
    lines.insert(b, f"\t\t{key} {val}")
    return b + 1


# ----------------------------------------------------------------------------- driver
@dataclass
class KernelMap:
    name: str
    insts: List[Inst]
    segments: List[List[int]]
    n_mem: int
    lds: int = 0              # static LDS bytes (group segment) of the original kernel
    vgprs: int = 32           # architected VGPRs per lane of the original kernel
    # (symbol, first instruction index, count) of each body in `insts`: the
    # kernel's own, then the device functions it may call (their PCs are
    # code-object addresses above FUNC_PC_BASE, so they never alias the
    # kernel's offsets in the simulator's instruction cache)
    parts: List[Tuple[str, int, int]] = field(default_factory=list)


FUNC_PC_BASE = 0x800000


def instrument(asm: str) -> Tuple[str, List[KernelMap]]:
    """Instrument every kernel of a gfx950 assembly file -- and every device
    function it may call -- and return the new assembly and the static map of
    each kernel.  A code object with device functions uses one probe register
    window for all of them (above every kernel's allocation, which covers its
    call graph), so a callee's probes find the state its caller's entry set
    up; function segments / memory records carry ids shared by every kernel."""
    lines = asm.split("\n")
    kernels = parse_kernels(lines)
    if not kernels:
        return asm, []
    fnames = function_names(lines) - set(kernels)
    funcs = parse_bodies(lines, fnames) if fnames else {}
    # descriptor facts and probe windows
    info: Dict[str, Dict] = {}
    for name in kernels:
        a, b = _descriptor_block(lines, name)
        nsg, _ = _dget(lines, a, b, ".amdhsa_next_free_sgpr")
        nvg, _ = _dget(lines, a, b, ".amdhsa_next_free_vgpr")
        acc, _ = _dget(lines, a, b, ".amdhsa_accum_offset", None)
        ucount, _ = _dget(lines, a, b, ".amdhsa_user_sgpr_count", 0)
        en = [(_dget(lines, a, b, f".amdhsa_system_sgpr_workgroup_id_{d}", 1 if d == "x" else 0)[0]) for d in "xyz"]
        winfo, _ = _dget(lines, a, b, ".amdhsa_system_sgpr_workgroup_info", 0)
        lds, _ = _dget(lines, a, b, ".amdhsa_group_segment_fixed_size", 0)
        S = max(nsg, ucount + 4)
        S += S & 1
        arch_v = acc if acc is not None and acc < nvg else nvg
        n_agpr = nvg - acc if acc is not None and acc < nvg else 0
        V = arch_v + (arch_v & 1)
        info[name] = dict(nsg=nsg, nvg=nvg, acc=acc, ucount=ucount, en=en, winfo=winfo, lds=lds, S=S, V=V,
                          arch_v=arch_v, n_agpr=n_agpr)
    if funcs:
        Sg = max(v["S"] for v in info.values())
        Vg = max(v["V"] for v in info.values())
        for v in info.values():
            v["S"], v["V"] = Sg, Vg
    for name, v in info.items():
        if v["S"] + N_PROBE_SGPR > MAX_SGPR:
            raise RewriteError(f"{name}: uses {v['nsg']} SGPRs, no room for the {N_PROBE_SGPR} probe SGPRs")
        if v["V"] + N_PROBE_VGPR > MAX_ARCH_VGPR:
            raise RewriteError(f"{name}: uses {v['arch_v']} VGPRs, no room for the {N_PROBE_VGPR} probe VGPRs")
    # segments: each kernel's own from 1, then the functions' from one base
    bodies: Dict[str, List[Tuple[int, str]]] = {}
    for name, k in kernels.items():
        bodies[name] = segment(k, lines)
        for ins in k.insts:
            if ins.mnem.startswith(("s_swappc", "s_call")) and not funcs:
                raise RewriteError(f"{name}: calls a device function that is not in this file")
            if ins.mnem.startswith("s_setpc"):
                raise RewriteError(f"{name}: indirect branch ({ins.text})")
    f0 = (max(len(k.segments) for k in kernels.values()) + 1) if funcs else 0
    m0 = max(k.n_mem for k in kernels.values()) if funcs else 0
    seg_next, mem_next = f0 - 1, m0
    forder = sorted(funcs, key=lambda n: funcs[n].start)
    for name in forder:
        f = funcs[name]
        bodies[name] = segment(f, lines, seg_next, mem_next)
        seg_next += len(f.segments)
        mem_next += f.n_mem
    # rebuild every body from the bottom so earlier line indices stay valid
    items = [(k.start, name, True) for name, k in kernels.items()] + [(f.start, name, False)
                                                                       for name, f in funcs.items()]
    ktag = {name: str(i) for i, name in enumerate(sorted(kernels, key=lambda n: -kernels[n].start))}
    ftag = {name: f"f{i}" for i, name in enumerate(forder)}
    for _, name, is_k in sorted(items, reverse=True):
        k = kernels[name] if is_k else funcs[name]
        if is_k:
            v = info[name]
            pr = Probe(v["S"], v["V"], ktag[name])
        else:
            pr = Probe(Sg, Vg, ftag[name])
        out: List[str] = []
        stubs: List[str] = []
        n = 0
        emitted_seg = 0
        if is_k:
            wg_sgprs = [v["ucount"], v["ucount"] + 1, v["ucount"] + 2]
            info_move = None
            if v["winfo"]:
                orig = v["ucount"] + sum(v["en"])
                if orig != v["ucount"] + 3:
                    info_move = (orig, v["ucount"] + 3)
            out += ["\t" + x if not x.endswith(":") else x for x in pr.entry(wg_sgprs, info_move)]
        for kind, ln in bodies[name]:
            if kind >= 0:
                ins = k.insts[kind]
                if ins.seg != emitted_seg:
                    emitted_seg = ins.seg
                    out += ["\t" + x if not x.endswith(":") else x for x in pr.segment(n, ins.seg, stubs)]
                    n += 1
                if ins.mem_id >= 0:
                    out += ["\t" + x if not x.endswith(":") else x for x in pr.memory(n, ins, stubs)]
                    n += 1
                if ins.mnem == "s_endpgm":
                    out += ["\t" + x if not x.endswith(":") else x for x in pr.close_at_end(n)]
                    n += 1
            out.append(ln)
        out += ["\t" + x if not x.endswith(":") else x for x in stubs]
        lines[k.start + 1:k.end] = out
        if not is_k:
            continue
        # descriptor (re-locate: the body above it changed size)
        S, V, acc, n_agpr = v["S"], v["V"], v["acc"], v["n_agpr"]
        a, b = _descriptor_block(lines, name)
        b = _dset(lines, a, b, ".amdhsa_next_free_sgpr", S + N_PROBE_SGPR)
        new_arch = V + N_PROBE_VGPR
        if acc is not None:
            new_acc = (new_arch + 3) // 4 * 4
            b = _dset(lines, a, b, ".amdhsa_accum_offset", new_acc)
            b = _dset(lines, a, b, ".amdhsa_next_free_vgpr", new_acc + n_agpr if n_agpr else new_arch)
        else:
            b = _dset(lines, a, b, ".amdhsa_next_free_vgpr", new_arch)
        for d in "xyz":
            b = _dset(lines, a, b, f".amdhsa_system_sgpr_workgroup_id_{d}", 1)
        # packed work-item ids (gfx90a+): x, y and z all land in v0
        b = _dset(lines, a, b, ".amdhsa_system_vgpr_workitem_id", 2)
        _fix_set_symbols(lines, name, S + N_PROBE_SGPR, new_arch)
    # maps: a kernel's own segments, then (ids f0..) every function's
    maps: List[KernelMap] = []
    for name in sorted(kernels, key=lambda n: kernels[n].start):
        k, v = kernels[name], info[name]
        insts = list(k.insts)
        segs = [list(sg) for sg in k.segments]
        parts = [(name, 0, len(k.insts))]
        if funcs:
            segs += [[] for _ in range(f0 - 1 - len(k.segments))]
            for fn in forder:
                f = funcs[fn]
                off = len(insts)
                parts.append((fn, off, len(f.insts)))
                insts += f.insts
                segs += [[off + i for i in sg] for sg in f.segments]
        maps.append(KernelMap(name, insts, segs, mem_next if funcs else k.n_mem, v["lds"], v["nvg"], parts))
    text = "\n".join(lines)
    text = _fix_metadata(text, {m.name for m in maps})
    text += _CTL_SYMBOL
    return text, maps


_CTL_SYMBOL = """
	.type	__asim_tctl,@object
	.section	.bss.__asim_tctl,"aw",@nobits
	.protected	__asim_tctl
	.globl	__asim_tctl
	.p2align	4, 0x0
__asim_tctl:
	.zero	32
	.size	__asim_tctl, 32
"""


def _fix_set_symbols(lines: List[str], name: str, nsgpr: int, nvgpr: int) -> None:
    for i, ln in enumerate(lines):
        s = ln.strip()
        for key, val in ((".num_vgpr", nvgpr), (".numbered_sgpr", nsgpr)):
            head = f".set {name}{key},"
            if s.startswith(head):
                expr = s[len(head):].strip()
                try:
                    lines[i] = f"\t{head} {max(int(expr, 0), val)}"
                except ValueError:  # a call graph's max(...) expression
                    lines[i] = f"\t{head} max({expr}, {val})"


def _fix_metadata(text: str, names: set) -> str:
    """raise .sgpr_count / .vgpr_count of instrumented kernels in the
    amdgpu_metadata YAML (informational for the runtime)."""
    i = text.find(".amdgpu_metadata")
    if i < 0:
        return text
    head, meta = text[:i], text[i:]
    blocks = re.split(r"(\n  - )", meta)
    out = [blocks[0]]
    for j in range(1, len(blocks), 2):
        sep, blk = blocks[j], blocks[j + 1]
        m = re.search(r"\.name:\s+(\S+)", blk)
        if m and m.group(1) in names:
            blk = re.sub(r"(\.sgpr_count:\s+)(\d+)", lambda g: g.group(1) + str(int(g.group(2)) + N_PROBE_SGPR + 4), blk)
            blk = re.sub(r"(\.vgpr_count:\s+)(\d+)", lambda g: g.group(1) + str(int(g.group(2)) + N_PROBE_VGPR + 2), blk)
        out += [sep, blk]
    return head + "".join(out)


# ----------------------------------------------------------------------------- static map
def assign_pcs(maps: Sequence[KernelMap], disasm: str) -> None:
    """Real byte offsets of each kernel's instructions from ``llvm-objdump -d``
    of the *uninstrumented* code object (instructions are 4 or 8 bytes)."""
    cur: Optional[List[int]] = None
    starts: Dict[str, List[int]] = {}
    base = 0
    for ln in disasm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:", ln)
        if m:
            base = int(m.group(1), 16)
            cur = starts.setdefault(m.group(2), [])
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+(\S+).*//\s*([0-9A-F]+):", ln)
        if m and not m.group(1).startswith("."):
            cur.append(int(m.group(2), 16) - base)
    for km in maps:
        # device functions: packed above FUNC_PC_BASE in their file order,
        # each at a 256 B boundary past the previous one's code (independent
        # of how the object laid them out, so a function recovered from a
        # linked binary gets the PCs its source-built twin gets)
        fbase = FUNC_PC_BASE
        for part, (sym, i0, n) in enumerate(km.parts or [(km.name, 0, len(km.insts))]):
            pcs = starts.get(sym)
            add = 0 if part == 0 else fbase
            if part:
                # the body's own instructions (the disassembly also lists the
                # alignment padding after it)
                fbase += ((pcs[n - 1] + 8 if pcs and len(pcs) >= n and n else 4 * n) + 255) // 256 * 256
            body = km.insts[i0:i0 + n]
            if pcs and len(pcs) >= len(body):
                for ins, pc in zip(body, pcs):
                    ins.pc = add + pc
            else:
                for i, ins in enumerate(body):
                    ins.pc = add + 4 * i


def trace_mnemonic(ins: Inst) -> str:
    """Trace opcode of an instruction: the mnemonic, with s_waitcnt's counts
    attached ('s_waitcnt.vm1.lgkm0'; a counter it does not name is not
    waited for) so the simulator can model count-based waits."""
    if ins.mnem != "s_waitcnt":
        return ins.mnem
    vm = re.search(r"vmcnt\((\d+)\)", ins.text)
    lg = re.search(r"lgkmcnt\((\d+)\)", ins.text)
    name = "s_waitcnt"
    if vm:
        name += f".vm{vm.group(1)}"
    if lg:
        name += f".lgkm{lg.group(1)}"
    if not vm and not lg:
        name += ".vm255.lgkm255" if "expcnt" in ins.text else ""
    return name


def write_map(maps: Sequence[KernelMap]) -> str:
    """Text map read by csrc/tracer/isa_runtime.cc."""
    out = [f"ASIMISA 1 {CHUNK_UNITS}"]
    for km in maps:
        out.append(f"K {km.name} {len(km.segments)} {km.n_mem} {km.lds} {km.vgprs}")
        for sid, idxs in enumerate(km.segments, start=1):
            out.append(f"S {sid} {len(idxs)}")
            for i in idxs:
                ins = km.insts[i]
                dst, src = reg_operands(ins)
                w = mem_width(ins.mnem) if ins.mem_id >= 0 else 0
                body = " ".join([str(len(dst))] + dst + [trace_mnemonic(ins), str(len(src))] + src)
                out.append(f"{ins.pc:x} {ins.mem_id} {body} {w}")
    return "\n".join(out) + "\n"
