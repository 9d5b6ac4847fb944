#!/usr/bin/env python3
"""Build a trace-capturing executable from unmodified HIP sources.

    python -m accel_sim_framework_distributed_amd.isatrace.build app.hip [more.hip] -o app.traced [-- hipcc flags]

Reference: the NVBit flow injects tracer_tool.so into an unmodified binary
(util/tracer_nvbit/run_hw_trace.py:51-121, tracer_tool.cu:130-275).  The
gfx950 flow instruments at the assembly level instead (no binary
instrumentation framework exists for CDNA4 in this stack):

1. ``hipcc -S --cuda-device-only`` -> the compiler's gfx950 assembly;
2. the uninstrumented assembly is assembled and disassembled once to learn
   every instruction's real byte offset (trace PCs);
3. isatrace.rewrite inserts the segment / memory probes, the assembly is
   assembled (clang -cc1as), linked (ld.lld) and bundled
   (clang-offload-bundler) into a fat binary;
4. the host side is compiled with that fat binary
   (``-fcuda-include-gpubinary``) and linked with the tracer runtime
   (csrc/tracer/isa_runtime.cc);
5. the static instruction map is written next to the executable
   (``<out>.asimisa``).

Running the result with ``ASIM_TRACE_DIR=<dir>`` writes kernel-N.traceg +
kernelslist.g; without it the program runs normally (the probes still
execute but the runtime does not arm the buffer -- the probes then find an
empty chunk pool and record nothing).
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import tempfile
from typing import List, Sequence

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.isatrace import binary, rewrite  # noqa: E402
else:
    from . import binary, rewrite

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LLVM = os.path.join(ROCM, "lib", "llvm", "bin")
ARCH = "gfx950"
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
RUNTIME_SRC = os.path.join(REPO, "csrc", "tracer", "isa_runtime.cc")


def _hipcc() -> str:
    return shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")


def _run(cmd: Sequence[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), file=sys.stderr)
    r = subprocess.run(list(cmd), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stderr[-4000:]}")


def runtime_object(work: str, verbose: bool = False) -> str:
    """The tracer runtime, compiled once per build directory."""
    obj = os.path.join(work, "isa_runtime.o")
    _run([_hipcc(), "-O2", "-fPIC", "-std=c++17", "-c", RUNTIME_SRC, "-o", obj], verbose)
    return obj


def instrument_source(src: str, work: str, flags: List[str], verbose: bool = False, device_from: str = ""):
    """Device half of one translation unit -> (fat binary path, kernel maps).
    With `device_from` (a precompiled host binary, shared library, bundle or
    code object) the device code is not compiled from `src`: the gfx950
    code object found there is turned back into assembly
    (isatrace/binary.py) and instrumented like compiler output -- the path
    for kernels whose sources are not at hand."""
    base = os.path.join(work, os.path.splitext(os.path.basename(src))[0])
    asm = base + ".s"
    if device_from:
        cos = binary.extract(device_from, os.path.join(work, "device_from"))
        if len(cos) != 1:
            raise RuntimeError(f"{device_from}: {len(cos)} gfx950 code objects (expected one)")
        lst = binary.disassemble(cos[0])
        bad = binary.unsupported(lst)
        if bad:
            raise RuntimeError(f"{device_from}: cannot instrument: " + "; ".join(bad[:5]))
        open(asm, "w").write(lst.asm())
    else:
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "--cuda-device-only", "-S", src, "-o", asm] + flags, verbose)
    text = open(asm).read()
    # real instruction offsets from the uninstrumented code object
    _run([os.path.join(LLVM, "clang"), "-target", "amdgcn-amd-amdhsa", f"-mcpu={ARCH}", "-c", asm, "-o",
          base + ".orig.o"], verbose)
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", base + ".orig.o"], stdout=subprocess.PIPE,
                         text=True, check=True).stdout
    new, maps = rewrite.instrument(text)
    rewrite.assign_pcs(maps, dis)
    open(base + ".instr.s", "w").write(new)
    _run([os.path.join(LLVM, "clang"), "-target", "amdgcn-amd-amdhsa", f"-mcpu={ARCH}", "-c", base + ".instr.s",
          "-o", base + ".instr.o"], verbose)
    _run([os.path.join(LLVM, "ld.lld"), "-shared", base + ".instr.o", "-o", base + ".co"], verbose)
    fb = base + ".hipfb"
    _run([os.path.join(LLVM, "clang-offload-bundler"), "-type=o", "-bundle-align=4096",
          f"-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--{ARCH}", "-input=/dev/null",
          f"-input={base}.co", f"-output={fb}"], verbose)
    return fb, maps


def build(sources: Sequence[str], out: str, flags: Sequence[str] = (), work: str = "", verbose: bool = False,
          libs: Sequence[str] = (), device_from: str = "") -> str:
    flags = list(flags)
    own = not work
    work = work or tempfile.mkdtemp(prefix="asim_isatrace_")
    os.makedirs(work, exist_ok=True)
    try:
        host_objs, all_maps = [], []
        for src in sources:
            fb, maps = instrument_source(src, work, flags, verbose, device_from)
            all_maps += maps
            ho = os.path.join(work, os.path.splitext(os.path.basename(src))[0] + ".host.o")
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "--cuda-host-only", "-Xclang",
                  "-fcuda-include-gpubinary", "-Xclang", fb, "-c", src, "-o", ho] + flags, verbose)
            host_objs.append(ho)
        rt = runtime_object(work, verbose)
        _run([_hipcc(), f"--offload-arch={ARCH}"] + host_objs + [rt, "-ldl"] + list(libs) + ["-o", out], verbose)
        with open(out + ".asimisa", "w") as f:
            f.write(rewrite.write_map(all_maps))
        return out
    finally:
        if own and not verbose:
            shutil.rmtree(work, ignore_errors=True)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    extra: List[str] = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("sources", nargs="+")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("-w", "--work_dir", default="", help="keep intermediate files here")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-L", "--libs", default="", help="extra link flags, e.g. '-lrccl'")
    ap.add_argument("--device-from", default="",
                    help="take the device code from this precompiled binary / code object instead of the source")
    o = ap.parse_args(argv)
    if o.device_from and len(o.sources) != 1:
        ap.error("--device-from needs exactly one source (its host half)")
    build(o.sources, o.out, extra, o.work_dir, o.verbose, o.libs.split(), o.device_from)
    print(f"built {o.out} (+ {o.out}.asimisa)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
