"""Precompiled code objects -> reassemblable gfx950 assembly (the binary-only
half of the automatic tracer).

Reference: the NVBit tracer instruments any SASS it finds at load time, library
kernels included (util/tracer_nvbit/tracer_tool/tracer_tool.cu:130-275,
380-506: every kernel a CUDA context launches, NCCL's included).  rewrite.py
instruments the compiler's own assembly, which needs the kernel's sources.
For a code object that ships without sources (a library's fat binary, a
hipModuleLoad'ed .hsaco) this module recovers an equivalent assembly file:

* ``extract(path)`` pulls the gfx950 code objects out of a host binary's or
  shared library's ``.hip_fatbin`` section (plain and compressed
  clang-offload-bundler bundles) or takes a raw code object;
* ``disassemble(co)`` lists every function with ``llvm-objdump
  --symbolize-operands`` (branch targets become labels), every kernel
  descriptor as the ``.amdhsa_kernel`` directives the disassembler decodes
  from its 64 bytes, the data sections (.rodata outside the descriptors,
  .data, .bss) as bytes with their symbols, and the ``NT_AMDGPU_METADATA``
  note as an ``.amdgpu_metadata`` block;
* PC-relative addresses -- ``s_getpc_b64 s[n:n+1]`` followed by ``s_add_u32
  sn, sn, lo`` / ``s_addc_u32 sn+1, sn+1, hi`` (direct calls to device
  functions, addresses of __constant__ / __device__ variables) -- become the
  compiler's own relocation form (``sym@rel32@lo+4`` / ``@hi+12``), so they
  stay right when the rewriter moves code; words of the data sections that
  the dynamic relocations fill (function / variable address tables) become
  ``.quad`` of their target symbol;
* ``roundtrip(co)`` assembles that listing again and compares every function
  (instruction bytes, the resolved targets of its PC-relative pairs), every
  kernel descriptor and every data object with the original: a code object
  is only handed to rewrite.py when its listing reproduces it.

What the listing cannot carry is refused, not guessed: a PC-relative pair
split by other instructions, a target outside every known symbol and
section, an indirect branch in a kernel that is not a resolved long branch.
``unsupported(lst)`` names them.  RCCL's gfx950 code object (126 kernels,
5.6k device functions, 20.6 M instructions): every one of its 8175
``s_getpc_b64`` triples is adjacent, its 8013 ``s_swappc_b64`` are direct
calls, its ``s_setpc_b64`` are returns or long branches -- nothing in it is
refused (``profiles/isatrace/rccl_census.json``).
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

LLVM = "/opt/rocm/lib/llvm/bin"
ARCH = "gfx950"
TRIPLE = "amdgcn-amd-amdhsa"
BUNDLE_TARGET = f"hipv4-{TRIPLE}--{ARCH}"
XNACK_SGPRS = 6  # SGPRs the assembler reserves for the XNACK mask (+ granule slack) on an xnack-"any" target

_FUNC_HDR = re.compile(r"^<([^>]+)>:\s*$")
_LABEL = re.compile(r"^<(L\d+)>:\s*$")
_INSN = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):((?:\s+[0-9A-Fa-f]{8})+)\s*$")
_GETPC = re.compile(r"^s_getpc_b64\s+s\[(\d+):(\d+)\]\s*$")
_ADD = re.compile(r"^s_add_u32\s+s(\d+),\s*s(\d+),\s*(\S+)\s*$")
_ADDC = re.compile(r"^s_addc_u32\s+s(\d+),\s*s(\d+),\s*(\S+)\s*$")
_SETPC = re.compile(r"^s_setpc_b64\s+s\[(\d+):(\d+)\]")
_DATA_SECTIONS = (".rodata", ".data", ".bss")


class BinaryError(RuntimeError):
    pass


def _run(cmd: List[str], **kw) -> str:
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, **kw)
    if p.returncode != 0:
        raise BinaryError(f"{' '.join(cmd[:3])} ...: {p.stderr.strip()[-800:]}")
    return p.stdout


def _is_code_object(path: str) -> bool:
    with open(path, "rb") as f:
        h = f.read(20)
    return len(h) == 20 and h[:4] == b"\x7fELF" and int.from_bytes(h[18:20], "little") == 224  # EM_AMDGPU


def extract(path: str, out_dir: str) -> List[str]:
    """gfx950 code objects of `path` (a raw code object, or a host binary /
    shared library with a .hip_fatbin section), written under out_dir."""
    os.makedirs(out_dir, exist_ok=True)
    if _is_code_object(path):
        return [path]
    with open(path, "rb") as f:
        head = f.read(24)
    if head.startswith((b"CCOB", b"__CLANG_OFFLOAD_BUNDLE__")):  # a bare bundle (.hipfb, hipcc -c device-only)
        fat = path
    else:
        fat = os.path.join(out_dir, "fatbin.bin")
        _run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", path,
              os.path.join(out_dir, "host.copy")])
        os.remove(os.path.join(out_dir, "host.copy"))
    # the section holds bundles back to back (each aligned): plain ones
    # ("__CLANG_OFFLOAD_BUNDLE__", sized by their entries) and compressed ones
    # ("CCOB" v2 / v3, whose header gives the total size); a plain bundle runs
    # to the next magic
    data = open(fat, "rb").read()
    spans = []
    pos = 0
    while pos < len(data):
        if data.startswith(b"CCOB", pos):
            ver = int.from_bytes(data[pos + 4:pos + 6], "little")
            total = (int.from_bytes(data[pos + 8:pos + 16], "little") if ver >= 3 else
                     int.from_bytes(data[pos + 8:pos + 12], "little") if ver == 2 else 0)
            if not total:
                raise BinaryError(f"{path}: compressed bundle v{ver} without a size field")
            spans.append((pos, pos + total))
            pos += total
        elif data.startswith(b"__CLANG_OFFLOAD_BUNDLE__", pos):
            nxt = [q for q in (data.find(b"CCOB", pos + 24), data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos + 24))
                   if q > 0]
            end = min(nxt) if nxt else len(data)
            spans.append((pos, end))
            pos = end
        else:  # alignment padding
            nz = len(data) - len(data[pos:].lstrip(b"\0"))
            pos = max(pos + 1, nz)
    outs = []
    for i, (s, e) in enumerate(spans):
        b = os.path.join(out_dir, f"bundle{i}.bin")
        with open(b, "wb") as f:
            f.write(data[s:e])
        targets = _run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={b}"]).split()
        if BUNDLE_TARGET not in targets:
            continue
        co = os.path.join(out_dir, f"bundle{i}.{ARCH}.co")
        _run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
              f"--targets={BUNDLE_TARGET}", f"--output={co}"])
        outs.append(co)
    return outs


# ----------------------------------------------------------------------- ELF
@dataclass
class Section:
    name: str
    addr: int
    off: int
    size: int
    nobits: bool
    align: int


@dataclass
class Sym:
    name: str
    addr: int
    size: int
    typ: str      # FUNC / OBJECT / NOTYPE
    bind: str     # GLOBAL / LOCAL / WEAK
    vis: str      # DEFAULT / PROTECTED / HIDDEN
    shndx: str


def _sections(co: str) -> Dict[str, Section]:
    out = {}
    for line in _run([f"{LLVM}/llvm-readelf", "-S", "--wide", co]).splitlines():
        m = re.match(r"\s*\[\s*\d+\]\s+(\S+)\s+(\S+)\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)\s+\S+\s+\S*\s+\d+\s+\d+\s+(\d+)",
                     line)
        if m:
            out[m.group(1)] = Section(m.group(1), int(m.group(3), 16), int(m.group(4), 16), int(m.group(5), 16),
                                      m.group(2) == "NOBITS", int(m.group(6)))
    return out


def _symbols(co: str) -> List[Sym]:
    out, seen = [], set()
    for line in _run([f"{LLVM}/llvm-readelf", "-s", "--wide", co]).splitlines():
        p = line.split()
        if len(p) < 8 or not p[0].rstrip(":").isdigit() or p[3] in ("FILE", "SECTION") or p[6] == "ABS":
            continue
        key = (p[7], int(p[1], 16))
        if key in seen:  # .symtab repeats .dynsym
            continue
        seen.add(key)
        out.append(Sym(p[7], int(p[1], 16), int(p[2]), p[3], p[4], p[5], p[6]))
    return out


def _relocs(co: str) -> Dict[int, Tuple[str, int, str]]:
    """Dynamic relocations: {offset: (type, addend, symbol or '')}."""
    out = {}
    for line in _run([f"{LLVM}/llvm-readelf", "-r", "--wide", co]).splitlines():
        p = line.split()
        if len(p) >= 3 and re.fullmatch(r"[0-9a-f]{16}", p[0]) and p[2].startswith("R_AMDGPU"):
            sym = p[4] if len(p) >= 6 and not p[4].startswith("+") else ""
            add = 0
            m = re.search(r"([+-])\s*([0-9a-f]+)\s*$", line)
            if m:
                add = int(m.group(2), 16) * (-1 if m.group(1) == "-" else 1)
            out[int(p[0], 16)] = (p[2], add, sym)
    return out


def _section_bytes(co: str, s: Section) -> bytes:
    if s.nobits:
        return bytes(s.size)
    with open(co, "rb") as f:
        f.seek(s.off)
        return f.read(s.size)


# ------------------------------------------------------------------- listing
@dataclass
class Func:
    name: str
    addr: int
    size: int
    kernel: bool
    lines: List[Tuple[str, int, bytes]] = field(default_factory=list)  # (text or label, addr, bytes)
    bind: str = "GLOBAL"
    vis: str = "DEFAULT"
    # PC-relative pairs: line index of the s_add / s_addc -> ("lo" | "hi", target address)
    pcrel: Dict[int, Tuple[str, int]] = field(default_factory=dict)
    bad: List[str] = field(default_factory=list)


@dataclass
class Listing:
    co: str
    funcs: List[Func]
    kds: Dict[str, str]          # kernel name -> .amdhsa_kernel block
    metadata: str                # YAML of the metadata note
    abi_version: int
    syms: List[Sym] = field(default_factory=list)
    sections: Dict[str, Section] = field(default_factory=dict)
    data: Dict[str, bytes] = field(default_factory=dict)      # data section -> bytes
    relocs: Dict[int, Tuple[str, int, str]] = field(default_factory=dict)

    # -- address -> symbolic name
    def _kd_ranges(self) -> List[Tuple[int, int]]:
        return [(s.addr, s.addr + 64) for s in self.syms if s.name.endswith(".kd")]

    def _insn_addrs(self) -> Dict[int, Tuple[int, str]]:
        out = {}
        for fi, f in enumerate(self.funcs):
            for text, a, _ in f.lines:
                if a >= 0:
                    out[a] = (fi, f.name)
        return out

    def symbolic(self, addr: int) -> Optional[str]:
        """A label expression for `addr`: a function or data symbol (+ offset),
        or the local label of an instruction / data byte."""
        for f in self.funcs:
            if f.addr == addr:
                return f.name
        for s in self.syms:
            if s.typ == "OBJECT" and not s.name.endswith(".kd") and s.addr <= addr < s.addr + max(1, s.size):
                return s.name if addr == s.addr else f"{s.name}+{addr - s.addr}"
        for f in self.funcs:
            if f.addr <= addr < f.addr + f.size:
                return f".Lt_{addr:x}"
        for n in _DATA_SECTIONS:
            s = self.sections.get(n)
            if s and s.addr <= addr < s.addr + max(1, s.size):
                return f".Ld_{addr:x}"
        return None

    def asm(self) -> str:
        """The whole code object as one assembly file."""
        cov = {2: 4, 3: 5, 4: 6}.get(self.abi_version, 5)
        out = [f'\t.amdgcn_target "{TRIPLE}--{ARCH}"', f"\t.amdhsa_code_object_version {cov}", "\t.text"]
        targets = set()
        for f in self.funcs:
            for _, (_, t) in f.pcrel.items():
                targets.add(t)
        for (_, add, _) in self.relocs.values():
            targets.add(add)
        tlabels = {t for t in targets if (self.symbolic(t) or "").startswith((".Lt_", ".Ld_"))}
        for fi, f in enumerate(self.funcs):
            if f.bind != "LOCAL":
                out.append(f"\t.globl {f.name}")
            if f.vis in ("PROTECTED", "HIDDEN"):
                out.append(f"\t.{f.vis.lower()} {f.name}")
            out += ["\t.p2align 8", f"\t.type {f.name},@function", f"{f.name}:"]
            for li, (text, a, _) in enumerate(f.lines):
                if text.startswith("<"):
                    out.append(f".Lb{fi}_{text[1:-2]}:")
                    continue
                if a in tlabels:
                    out.append(f".Lt_{a:x}:")
                if li in f.pcrel:
                    part, t = f.pcrel[li]
                    ops = text.rsplit(",", 1)[0]
                    text = f"{ops}, {self.symbolic(t)}@rel32@{part}+{4 if part == 'lo' else 12}"
                out.append("\t" + re.sub(r"\b(L\d+)\b", lambda m: f".Lb{fi}_{m.group(1)}", text))
            out.append(f".Lfunc_end{fi}:")
            out.append(f"\t.size {f.name}, .Lfunc_end{fi}-{f.name}")
        out.append("\t.rodata")
        for name, kd in self.kds.items():
            out += ["\t.p2align 6", kd]
        out += self._data_asm(tlabels)
        out += ["\t.amdgpu_metadata", self.metadata.rstrip(), "\t.end_amdgpu_metadata", ""]
        return "\n".join(out)

    def _data_asm(self, tlabels) -> List[str]:
        out = []
        kd = self._kd_ranges()
        objs = sorted((s for s in self.syms if s.typ in ("OBJECT", "NOTYPE") and not s.name.endswith(".kd")
                       and not s.name.startswith("_DYNAMIC")), key=lambda s: s.addr)
        for n in _DATA_SECTIONS:
            s = self.sections.get(n)
            if not s or not s.size:
                continue
            raw = self.data[n]
            here = [o for o in objs if s.addr <= o.addr < s.addr + s.size]
            out.append(f"\t.section {n}" if n != ".rodata" else "\t.rodata")
            # every byte outside the kernel descriptors, in address order
            a = s.addr
            end = s.addr + s.size
            first = True
            while a < end:
                r = next(((lo, hi) for lo, hi in kd if lo <= a < hi), None)
                if r:
                    a = r[1]
                    first = True
                    continue
                if first:  # keep the original alignment of every run
                    al = min(s.align, a & -a if a else s.align) or 1
                    out.append(f"\t.p2align {max(0, al.bit_length() - 1)}")
                    first = False
                for o in here:
                    if o.addr == a:
                        if o.bind != "LOCAL":
                            out.append(f"\t.globl {o.name}")
                        if o.vis in ("PROTECTED", "HIDDEN"):
                            out.append(f"\t.{o.vis.lower()} {o.name}")
                        out += [f"\t.type {o.name},@object", f"\t.size {o.name}, {o.size}", f"{o.name}:"]
                if a in tlabels:
                    out.append(f".Ld_{a:x}:")
                rel = self.relocs.get(a)
                if rel and rel[0] in ("R_AMDGPU_RELATIVE64", "R_AMDGPU_ABS64"):
                    tgt = rel[2] if rel[2] else self.symbolic(rel[1])
                    out.append(f"\t.quad {tgt}" + (f"+{rel[1]}" if rel[2] and rel[1] else ""))
                    a += 8
                    continue
                # run of plain bytes up to the next symbol / label / relocation / descriptor
                stops = [o.addr for o in here if o.addr > a] + [t for t in tlabels if a < t < end] + \
                        [r0 for r0 in self.relocs if a < r0 < end] + [lo for lo, _ in kd if a < lo < end] + [end]
                b = min(stops)
                chunk = raw[a - s.addr:b - s.addr]
                if s.nobits or not any(chunk):
                    out.append(f"\t.zero {b - a}")
                else:
                    for i in range(0, len(chunk), 32):
                        out.append("\t.byte " + ",".join(str(x) for x in chunk[i:i + 32]))
                a = b
        return out


def _kd_for_assembler(kd: str) -> str:
    """The decoded descriptor in the form the assembler reproduces: the
    decoder prints the SGPR granule's full count with the XNACK mask
    reservation folded in, while for an xnack-"any" target the assembler adds
    that reservation itself (and refuses the directive): take it out of
    next_free_sgpr and drop the directive."""
    out = []
    for l in kd.splitlines():
        if ".amdhsa_reserve_xnack_mask" in l:
            continue
        m = re.match(r"(\s*\.amdhsa_next_free_sgpr\s+)(\d+)", l)
        if m:
            l = f"{m.group(1)}{max(0, int(m.group(2)) - XNACK_SGPRS)}"
        out.append(l)
    return "\n".join(out)


def _literal(op: str) -> Optional[int]:
    try:
        return int(op, 0) & 0xFFFFFFFF
    except ValueError:
        return None


def _resolve_pcrel(f: Func) -> None:
    """Find the s_getpc_b64 / s_add_u32 / s_addc_u32 triples (adjacent, as
    the compiler emits them) and record their targets."""
    insns = [(i, t, a) for i, (t, a, _) in enumerate(f.lines) if a >= 0]
    for k, (i, t, a) in enumerate(insns):
        m = _GETPC.match(t)
        if not m:
            continue
        lo_r, hi_r = int(m.group(1)), int(m.group(2))
        nxt = insns[k + 1:k + 3]
        ok = len(nxt) == 2
        if ok:
            (i1, t1, a1), (i2, t2, a2) = nxt
            m1, m2 = _ADD.match(t1), _ADDC.match(t2)
            ok = (m1 and m2 and int(m1.group(1)) == lo_r == int(m1.group(2)) and
                  int(m2.group(1)) == hi_r == int(m2.group(2)) and a1 == a + 4 and a2 == a + 12)
        if not ok:
            f.bad.append(f"{f.name}+{a - f.addr:#x}: s_getpc_b64 not followed by its s_add_u32 / s_addc_u32 pair")
            continue
        lo, hi = _literal(m1.group(3)), _literal(m2.group(3))
        if lo is None or hi is None:
            continue  # already symbolic
        off = (hi << 32) | lo
        if off >> 63:
            off -= 1 << 64
        tgt = a + 4 + off
        f.pcrel[i1] = ("lo", tgt)
        f.pcrel[i2] = ("hi", tgt)


def disassemble(co: str) -> Listing:
    syms = _symbols(co)
    secs = _sections(co)
    kernels = {s.name[:-3] for s in syms if s.typ == "OBJECT" and s.name.endswith(".kd")}
    fsyms = sorted((s for s in syms if s.typ == "FUNC" and s.size), key=lambda s: s.addr)
    text = _run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", "--no-show-raw-insn", "--no-leading-addr",
                 f"--mcpu={ARCH}", co])
    funcs = [Func(s.name, s.addr, s.size, s.name in kernels, bind=s.bind, vis=s.vis) for s in fsyms]
    by_name: Dict[str, Func] = {f.name: f for f in funcs}
    cur: Optional[Func] = None
    for line in text.splitlines():
        m = _LABEL.match(line)
        if m:
            if cur is not None:
                cur.lines.append((f"<{m.group(1)}>:", -1, b""))
            continue
        m = _FUNC_HDR.match(line)
        if m:
            cur = by_name.get(m.group(1))
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if m:
            addr = int(m.group(2), 16)
            if cur.addr <= addr < cur.addr + cur.size:
                raw = b"".join(int(w, 16).to_bytes(4, "little") for w in m.group(3).split())
                cur.lines.append((m.group(1), addr, raw))
    for f in funcs:
        _resolve_pcrel(f)
    kds = {}
    for k in sorted(kernels, key=lambda n: next(s.addr for s in syms if s.name == n + ".kd")):
        d = _run([f"{LLVM}/llvm-objdump", "-D", f"--mcpu={ARCH}", f"--disassemble-symbols={k}.kd", co])
        i, j = d.find(".amdhsa_kernel"), d.find(".end_amdhsa_kernel")
        if i < 0 or j < 0:
            raise BinaryError(f"{co}: kernel descriptor of {k} not decoded")
        kd = _kd_for_assembler(d[i:j + len(".end_amdhsa_kernel")])
        if ".amdhsa_user_sgpr_count" not in kd:
            # the decoder leaves the user-SGPR count implicit; the rewriter
            # needs it to find the workgroup-id SGPRs: COMPUTE_PGM_RSRC2
            # (descriptor byte 52) bits 1-5
            ksym = next(s for s in syms if s.name == k + ".kd")
            ro = secs[".rodata"]
            rsrc2 = int.from_bytes(_section_bytes(co, ro)[ksym.addr - ro.addr + 52:ksym.addr - ro.addr + 56], "little")
            head, rest = kd.split("\n", 1)
            kd = f"{head}\n\t.amdhsa_user_sgpr_count {(rsrc2 >> 1) & 31}\n{rest}"
        kds[k] = kd
    notes = _run([f"{LLVM}/llvm-readelf", "--notes", co])
    i = notes.find("---")
    j = notes.find("\n...", i)
    if i < 0:
        raise BinaryError(f"{co}: no AMDGPU metadata note")
    meta = notes[i:j + 4]  # readelf indents only the document marker
    # the descriptor holds register counts rounded to the allocation granule;
    # the metadata note keeps the compiler's exact ones (what the traces'
    # "-nregs" and the rewriter's probe registers are derived from)
    for blk in re.split(r"\n  - ", meta)[1:]:
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or m.group(1) not in kds:
            continue
        sg = re.search(r"\.sgpr_count:\s+(\d+)", blk)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        ag = re.search(r"\.agpr_count:\s+(\d+)", blk)
        kd = kds[m.group(1)]
        if sg:
            kd = re.sub(r"(\.amdhsa_next_free_sgpr\s+)\d+", lambda g: f"{g.group(1)}{max(0, int(sg.group(1)) - XNACK_SGPRS)}", kd)
        if vg and (not ag or int(ag.group(1)) == 0):
            kd = re.sub(r"(\.amdhsa_next_free_vgpr\s+)\d+", lambda g: f"{g.group(1)}{vg.group(1)}", kd)
        kds[m.group(1)] = kd
    abi = 0
    for line in _run([f"{LLVM}/llvm-readelf", "-h", co]).splitlines():
        if "ABI Version" in line:
            abi = int(line.split()[-1])
    data = {n: _section_bytes(co, secs[n]) for n in _DATA_SECTIONS if n in secs}
    return Listing(co, funcs, kds, meta, abi, syms, secs, data, _relocs(co))


def unsupported(lst: Listing) -> List[str]:
    """Constructs the listing cannot carry through instrumentation."""
    bad = []
    for f in lst.funcs:
        bad += f.bad
        for _, (part, t) in sorted(f.pcrel.items()):
            if part == "lo" and lst.symbolic(t) is None:
                bad.append(f"{f.name}: PC-relative target {t:#x} outside every symbol and section")
        # s_setpc_b64 is a device function's return (s[30:31], or wherever
        # the function moved its return address) or a long branch whose
        # target came from an s_getpc_b64 triple right before it (resolved
        # above, the target gets a label); in a kernel only the latter
        insns = [(t, a) for t, a, _ in f.lines if a >= 0]
        for k, (text, a) in enumerate(insns):
            m = _SETPC.match(text)
            if not m:
                continue
            g = _GETPC.match(insns[k - 3][0]) if k >= 3 else None
            long_branch = g is not None and (g.group(1), g.group(2)) == (m.group(1), m.group(2))
            if f.kernel and not long_branch:
                bad.append(f"{f.name}+{a - f.addr:#x}: indirect branch ({text})")
    return bad


def assemble(asm: str, out: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "in.s")
        o = os.path.join(td, "in.o")
        with open(s, "w") as f:
            f.write(asm)
        _run([f"{LLVM}/clang", "-x", "assembler", "-target", TRIPLE, f"-mcpu={ARCH}", "-c", s, "-o", o])
        _run([f"{LLVM}/ld.lld", "-shared", o, "-o", out])
    return out


def _insn_bytes(f: Func) -> bytes:
    """A function's machine code with the PC-relative literals blanked (they
    move with the layout; their targets are compared symbolically)."""
    skip = set(f.pcrel)
    return b"".join(r[:4] if i in skip else r for i, (_, a, r) in enumerate(f.lines) if a >= 0)


def roundtrip(co: str, work: str) -> Dict:
    """Disassemble, reassemble and compare every function, descriptor and
    data object."""
    lst = disassemble(co)
    os.makedirs(work, exist_ok=True)
    out = assemble(lst.asm(), os.path.join(work, "roundtrip.co"))
    back = disassemble(out)
    res = {"functions": len(lst.funcs), "kernels": sum(f.kernel for f in lst.funcs), "identical": 0,
           "mismatch": [], "pcrel": sum(len(f.pcrel) // 2 for f in lst.funcs), "unsupported": unsupported(lst)}
    other = {f.name: f for f in back.funcs}
    for f in lst.funcs:
        g = other.get(f.name)
        same = g is not None and _insn_bytes(f) == _insn_bytes(g)
        if same:
            t1 = [lst.symbolic(t) for _, (p, t) in sorted(f.pcrel.items()) if p == "lo"]
            t2 = [back.symbolic(t) for _, (p, t) in sorted(g.pcrel.items()) if p == "lo"]
            same = t1 == t2
        if same:
            res["identical"] += 1
        else:
            res["mismatch"].append(f.name)
    res["kd_identical"] = all(back.kds.get(k) == v for k, v in lst.kds.items())
    # data objects: bytes, except words a relocation fills (compared by target)
    bo = {s.name: s for s in back.syms}
    bad_obj = []
    for s in lst.syms:
        if s.typ != "OBJECT" or s.name.endswith(".kd") or not s.size or s.name not in bo:
            continue
        def obj_bytes(L: Listing, sym: Sym) -> bytes:
            for n, sec in L.sections.items():
                if n in L.data and sec.addr <= sym.addr < sec.addr + sec.size:
                    b = bytearray(L.data[n][sym.addr - sec.addr:sym.addr - sec.addr + sym.size])
                    for r in L.relocs:
                        if sym.addr <= r < sym.addr + sym.size:
                            b[r - sym.addr:r - sym.addr + 8] = bytes(8)
                    return bytes(b)
            return b""
        if obj_bytes(lst, s) != obj_bytes(back, bo[s.name]):
            bad_obj.append(s.name)
    res["data_identical"] = not bad_obj
    res["data_mismatch"] = bad_obj
    return res


__all__ = ["extract", "disassemble", "assemble", "roundtrip", "unsupported", "Listing", "Func", "BinaryError"]
