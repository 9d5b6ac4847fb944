"""Trace file formats (Python side).

* ``.asimk`` -- this project's binary columnar kernel trace (layout mirrors
  ``csrc/trace/trace.cc`` ``BinHdr`` + ``TInst``/``TMem``/``WStream`` arrays).
  Config independent: coalescing happens at load time in the simulator.
* ``kernelslist.g`` + ``kernel-N.traceg`` -- the reference's text formats
  (trace_parser.cc:220-447), written for compatibility tests and tools.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterable, List, Sequence

import numpy as np

# ---- op classes (csrc/model/types.h OpCls) ----
OC = dict(ALU=0, SP=1, DP=2, SFU=3, TENSOR=4, INTP=5, LOAD=6, STORE=7, BRANCH=8, BARRIER=9,
          MEMBAR=10, EXIT=11, NOP=12, SPEC1=13, SPEC2=14, SPEC3=15)
SPACE = dict(NONE=0, GLOBAL=1, LOCAL=2, SHARED=3, CONST=4, TEX=5, PARAM=6)
FLAG = dict(BYPASS_L1=1, ATOMIC=2, MEM=4, WAITCNT=8)
NO_MEM = 0xFFFFFFFF

TINST = np.dtype([("pc", "<u4"), ("mem", "<u4"), ("mask", "<u8"), ("opcode", "<u2"), ("cls", "u1"),
                  ("space", "u1"), ("dst", "u1", (2,)), ("src", "u1", (5,)), ("width", "u1"),
                  ("lat", "<u2"), ("ii", "u1"), ("flags", "u1")])
TMEM = np.dtype([("base", "<u8"), ("stride", "<i4"), ("list", "<u4")])
WSTREAM = np.dtype([("begin", "<u4"), ("count", "<u4")])
assert TINST.itemsize == 32 and TMEM.itemsize == 16 and WSTREAM.itemsize == 8

_HDR = struct.Struct("<8sII3I3IIIQIIQQIIIIQQQQQ")
MAGIC = b"ASIMK001"

# SASS mnemonic -> (class, space, flags, width) for the opcodes the generators emit
SASS = {
    "IMAD": ("INTP", "NONE", 0, 0), "IADD3": ("INTP", "NONE", 0, 0), "ISETP": ("INTP", "NONE", 0, 0),
    "LOP3": ("INTP", "NONE", 0, 0), "SHF": ("INTP", "NONE", 0, 0), "LEA": ("INTP", "NONE", 0, 0),
    "IMAD.WIDE": ("INTP", "NONE", 0, 0), "IMNMX": ("INTP", "NONE", 0, 0),
    "MOV": ("ALU", "NONE", 0, 0), "S2R": ("ALU", "NONE", 0, 0), "SEL": ("ALU", "NONE", 0, 0),
    "LDC": ("ALU", "CONST", 0, 0), "SHFL.BFLY": ("ALU", "NONE", 0, 0), "CS2R": ("ALU", "NONE", 0, 0),
    "FFMA": ("SP", "NONE", 0, 0), "FADD": ("SP", "NONE", 0, 0), "FMUL": ("SP", "NONE", 0, 0),
    "FSETP": ("SP", "NONE", 0, 0), "FMNMX": ("SP", "NONE", 0, 0), "FSEL": ("SP", "NONE", 0, 0),
    "HFMA2": ("SP", "NONE", 0, 0),
    "DFMA": ("DP", "NONE", 0, 0), "DADD": ("DP", "NONE", 0, 0), "DMUL": ("DP", "NONE", 0, 0),
    "MUFU.RCP": ("SFU", "NONE", 0, 0), "MUFU.SQRT": ("SFU", "NONE", 0, 0), "MUFU.EX2": ("SFU", "NONE", 0, 0),
    "MUFU.LG2": ("SFU", "NONE", 0, 0), "MUFU.RSQ": ("SFU", "NONE", 0, 0),
    "HMMA.1688.F32": ("SPEC3", "NONE", 0, 0), "HMMA.884.F32.F32.STEP0": ("SPEC3", "NONE", 0, 0),
    "HMMA.884.F32.F32.STEP1": ("SPEC3", "NONE", 0, 0),
    "BRA": ("SPEC1", "NONE", 0, 0), "BSSY": ("SPEC1", "NONE", 0, 0), "BSYNC": ("SPEC1", "NONE", 0, 0),
    "BAR.SYNC": ("BARRIER", "NONE", 0, 0), "MEMBAR.GL": ("MEMBAR", "NONE", 0, 0),
    "EXIT": ("EXIT", "NONE", 0, 0), "NOP": ("NOP", "NONE", 0, 0),
    "LDG.E": ("LOAD", "GLOBAL", FLAG["MEM"], 4), "LDG.E.64": ("LOAD", "GLOBAL", FLAG["MEM"], 8),
    "LDG.E.128": ("LOAD", "GLOBAL", FLAG["MEM"], 16),
    "LDG.E.CONSTANT": ("LOAD", "GLOBAL", FLAG["MEM"], 4),
    "STG.E": ("STORE", "GLOBAL", FLAG["MEM"], 4), "STG.E.64": ("STORE", "GLOBAL", FLAG["MEM"], 8),
    "STG.E.128": ("STORE", "GLOBAL", FLAG["MEM"], 16), "STG.E.U16": ("STORE", "GLOBAL", FLAG["MEM"], 2),
    "LDL": ("LOAD", "LOCAL", FLAG["MEM"], 4), "STL": ("STORE", "LOCAL", FLAG["MEM"], 4),
    "LDS": ("LOAD", "SHARED", FLAG["MEM"], 4), "LDS.64": ("LOAD", "SHARED", FLAG["MEM"], 8),
    "STS": ("STORE", "SHARED", FLAG["MEM"], 4), "STS.64": ("STORE", "SHARED", FLAG["MEM"], 8),
    "LDS.128": ("LOAD", "SHARED", FLAG["MEM"], 16), "STS.128": ("STORE", "SHARED", FLAG["MEM"], 16),
    "ATOMG.E.ADD.STRONG.GPU": ("LOAD", "GLOBAL", FLAG["MEM"] | FLAG["ATOMIC"] | FLAG["BYPASS_L1"], 4),
    "RED.E.ADD.STRONG.GPU": ("LOAD", "GLOBAL", FLAG["MEM"] | FLAG["ATOMIC"] | FLAG["BYPASS_L1"], 4),
    "ATOMS.ADD": ("LOAD", "SHARED", FLAG["MEM"], 4),
}


# CDNA4 (gfx950) mnemonics for native wave64 traces; classes follow the
# simulator's CDNA decoder (csrc/trace/trace.cc decode_cdna)
CDNA = {
    "v_fma_f32": ("SP", "NONE", 0, 0), "v_add_f32": ("SP", "NONE", 0, 0), "v_mul_f32": ("SP", "NONE", 0, 0),
    "v_mov_b32": ("SP", "NONE", 0, 0), "v_mad_u32_u24": ("SP", "NONE", 0, 0), "v_add_u32": ("SP", "NONE", 0, 0),
    "v_mul_lo_u32": ("SP", "NONE", 0, 0), "v_lshlrev_b32": ("SP", "NONE", 0, 0), "v_cmp_gt_i32": ("SP", "NONE", 0, 0),
    "v_fma_f64": ("DP", "NONE", 0, 0), "v_add_f64": ("DP", "NONE", 0, 0),
    "v_sqrt_f32": ("SFU", "NONE", 0, 0), "v_exp_f32": ("SFU", "NONE", 0, 0), "v_rcp_f32": ("SFU", "NONE", 0, 0),
    "v_mfma_f32_32x32x16_bf16": ("TENSOR", "NONE", 0, 0),
    "s_add_u32": ("INTP", "NONE", 0, 0), "s_mul_i32": ("INTP", "NONE", 0, 0), "s_cmp_lt_i32": ("INTP", "NONE", 0, 0),
    "s_cbranch_scc1": ("BRANCH", "NONE", 0, 0), "s_branch": ("BRANCH", "NONE", 0, 0),
    "s_waitcnt": ("NOP", "NONE", FLAG["WAITCNT"], 0), "s_barrier": ("BARRIER", "NONE", 0, 0),
    "s_load_dwordx2": ("LOAD", "CONST", 0, 8), "s_load_dwordx4": ("LOAD", "CONST", 0, 16),
    "s_endpgm": ("EXIT", "NONE", 0, 0), "s_nop": ("NOP", "NONE", 0, 0),
    "global_load_dword": ("LOAD", "GLOBAL", FLAG["MEM"], 4), "global_load_dwordx2": ("LOAD", "GLOBAL", FLAG["MEM"], 8),
    "global_load_dwordx4": ("LOAD", "GLOBAL", FLAG["MEM"], 16),
    "global_store_dword": ("STORE", "GLOBAL", FLAG["MEM"], 4),
    "global_store_dwordx4": ("STORE", "GLOBAL", FLAG["MEM"], 16),
    "global_atomic_add": ("LOAD", "GLOBAL", FLAG["MEM"] | FLAG["ATOMIC"] | FLAG["BYPASS_L1"], 4),
    "ds_read_b32": ("LOAD", "SHARED", FLAG["MEM"], 4), "ds_write_b32": ("STORE", "SHARED", FLAG["MEM"], 4),
    "ds_read_b64": ("LOAD", "SHARED", FLAG["MEM"], 8), "ds_read_b128": ("LOAD", "SHARED", FLAG["MEM"], 16),
    "ds_write_b64": ("STORE", "SHARED", FLAG["MEM"], 8), "ds_write_b128": ("STORE", "SHARED", FLAG["MEM"], 16),
}


def op_info(mnemonic: str):
    table = SASS if mnemonic in SASS else CDNA
    if mnemonic not in table:
        raise KeyError(f"generator does not know opcode {mnemonic!r}")
    c, s, f, w = table[mnemonic]
    return OC[c], SPACE[s], f, w


class KernelArrays:
    """Plain container of one decoded kernel trace."""

    def __init__(self, header: Dict, insts: np.ndarray, mems: np.ndarray, addrs: np.ndarray,
                 streams: np.ndarray, opnames: Sequence[str]):
        self.header = header
        self.insts = insts
        self.mems = mems
        self.addrs = addrs
        self.streams = streams
        self.opnames = list(opnames)

    @property
    def thread_insts(self) -> int:
        m = np.ascontiguousarray(self.insts["mask"])
        return int(np.unpackbits(m.view(np.uint8)).sum()) if len(m) else 0


def write_kernel_binary(path: str, k: KernelArrays) -> None:
    h = k.header
    name = h["name"].encode()
    grid = list(h["grid"]) + [1] * (3 - len(h["grid"]))
    block = list(h["block"]) + [1] * (3 - len(h["block"]))
    ws = int(h.get("warp_size", 32))
    wpc = -(-int(np.prod(block)) // ws)
    ncta = int(np.prod(grid))
    assert len(k.streams) == ncta * wpc, "streams must be [n_cta * warps_per_cta]"
    hdr = _HDR.pack(MAGIC, 1, int(h.get("id", 1)), *grid, *block, int(h.get("shmem", 0)), int(h.get("nregs", 32)),
                    int(h.get("stream", 0)), int(h.get("binary_version", 70)), int(h.get("trace_version", 4)),
                    int(h.get("shmem_base", 0x00007f0000000000)), int(h.get("local_base", 0x00007f1000000000)),
                    ws, wpc, ncta, len(name), len(k.insts), len(k.mems), len(k.addrs), len(k.streams),
                    k.thread_insts)
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(name)
        used = sorted(set(int(x) for x in np.unique(k.insts["opcode"]))) if len(k.insts) else []
        f.write(struct.pack("<I", len(used)))
        for i in used:
            nm = k.opnames[i].encode()
            f.write(struct.pack("<HH", i, len(nm)))
            f.write(nm)
        f.write(np.ascontiguousarray(k.insts, TINST).tobytes())
        f.write(np.ascontiguousarray(k.mems, TMEM).tobytes())
        f.write(np.ascontiguousarray(k.addrs, np.uint64).tobytes())
        f.write(np.ascontiguousarray(k.streams, WSTREAM).tobytes())


def read_kernel_binary(path: str) -> KernelArrays:
    with open(path, "rb") as f:
        raw = f.read()
    fields = _HDR.unpack_from(raw, 0)
    if fields[0] != MAGIC:
        raise ValueError(f"{path}: not an .asimk file")
    (_, _ver, kid, gx, gy, gz, bx, by, bz, shmem, nregs, stream, bv, tv, sbase, lbase, ws, wpc, ncta, nlen,
     ni, nm, na, ns, _ti) = fields
    off = _HDR.size
    name = raw[off:off + nlen].decode()
    off += nlen
    (nu,) = struct.unpack_from("<I", raw, off)
    off += 4
    opnames: Dict[int, str] = {}
    for _ in range(nu):
        i, ln = struct.unpack_from("<HH", raw, off)
        off += 4
        opnames[i] = raw[off:off + ln].decode()
        off += ln
    insts = np.frombuffer(raw, TINST, ni, off).copy()
    off += ni * TINST.itemsize
    mems = np.frombuffer(raw, TMEM, nm, off).copy()
    off += nm * TMEM.itemsize
    addrs = np.frombuffer(raw, np.uint64, na, off).copy()
    off += na * 8
    streams = np.frombuffer(raw, WSTREAM, ns, off).copy()
    names = [""] * (max(opnames) + 1 if opnames else 1)
    for i, n in opnames.items():
        names[i] = n
    header = dict(name=name, id=kid, grid=(gx, gy, gz), block=(bx, by, bz), shmem=shmem, nregs=nregs,
                  stream=stream, binary_version=bv, trace_version=tv, shmem_base=sbase, local_base=lbase,
                  warp_size=ws)
    return KernelArrays(header, insts, mems, addrs, streams, names)


def write_kernel_text(path: str, k: KernelArrays) -> None:
    """Reference-compatible ``.traceg`` text (v4, post-processed, grouped by TB)."""
    h = k.header
    grid = list(h["grid"])
    block = list(h["block"])
    ws = int(h.get("warp_size", 32))
    wpc = -(-int(np.prod(block)) // ws)
    lines = [f"-kernel name = {h['name']}", f"-kernel id = {h.get('id', 1)}",
             f"-grid dim = ({grid[0]},{grid[1]},{grid[2]})", f"-block dim = ({block[0]},{block[1]},{block[2]})",
             f"-shmem = {h.get('shmem', 0)}", f"-nregs = {h.get('nregs', 32)}",
             f"-binary version = {h.get('binary_version', 70)}", f"-cuda stream id = {h.get('stream', 0)}",
             f"-shmem base_addr = 0x{h.get('shmem_base', 0x00007f0000000000):016x}",
             f"-local mem base_addr = 0x{h.get('local_base', 0x00007f1000000000):016x}",
             "-nvbit version = 1.5.5", f"-accelsim tracer version = {h.get('trace_version', 4)}"]
    if ws != 32:
        lines.append(f"-warp size = {ws}")
    lines += ["", "#traces format = threadblock_x threadblock_y threadblock_z warpid_tb PC mask dest_num "
              "reg_dests opcode src_num reg_srcs mem_width [adrrescompress?] [mem_addresses]", ""]
    out = ["\n".join(lines)]
    ncta = int(np.prod(grid))
    for c in range(ncta):
        x, y, z = c % grid[0], (c // grid[0]) % grid[1], c // (grid[0] * grid[1])
        buf = ["#BEGIN_TB", "", f"thread block = {x},{y},{z}", ""]
        for w in range(wpc):
            s = k.streams[c * wpc + w]
            b, n = int(s["begin"]), int(s["count"])
            buf.append(f"warp = {w}")
            buf.append(f"insts = {n}")
            for i in range(b, b + n):
                it = k.insts[i]
                dst = [f"R{int(r) - 1}" for r in it["dst"] if r]
                src = [f"R{int(r) - 1}" for r in it["src"] if r]
                parts = [f"{int(it['pc']):04x}", f"{int(it['mask']):08x}", str(len(dst)), *dst,
                         k.opnames[int(it["opcode"])], str(len(src)), *src]
                if int(it["mem"]) != NO_MEM:
                    m = k.mems[int(it["mem"])]
                    parts.append(str(int(it["width"])))
                    if int(m["list"]) == NO_MEM:
                        parts += ["1", f"0x{int(m['base']):x}", str(int(m["stride"]))]
                    else:
                        n_act = bin(int(it["mask"])).count("1")
                        lst = k.addrs[int(m["list"]):int(m["list"]) + n_act]
                        parts += ["0"] + [f"0x{int(a):x}" for a in lst]
                else:
                    parts.append("0")
                buf.append(" ".join(parts))
            buf.append("")
        buf += ["#END_TB", ""]
        out.append("\n".join(buf))
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def write_kernelslist(dirpath: str, commands: Iterable[str], name: str = "kernelslist.g") -> str:
    p = os.path.join(dirpath, name)
    with open(p, "w") as f:
        for c in commands:
            f.write(c + "\n")
    return p
