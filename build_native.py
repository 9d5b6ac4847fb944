#!/usr/bin/env python3
"""Build the native parts in-tree (no installation).

Outputs
  accel_sim_framework_distributed_amd/_asim*.so   pybind11 module (CPU + HIP engines)
  bin/accel-sim.out                               accel-sim compatible CLI
  bin/ubench/*                                    HIP micro-benchmarks (gfx950)
  bin/libasim_tracer.so                           rocprofiler-sdk trace capture tool

Host C++ is compiled with g++ (OpenMP for the CPU engine), device code with
``hipcc --offload-arch=gfx950``.  A ninja file is generated under build/ so
incremental rebuilds are fast.  Usage: ``python build_native.py [--cpu-only] [-j N]``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "accel_sim_framework_distributed_amd")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
# apps whose traced twin is also built from the precompiled binary alone (bin/isatrace_bin)
BINARY_PATH_APPS = ("nw", "lud", "hotspot", "backprop", "devcalls")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

CORE_SRC = [
    "csrc/config/options.cc",
    "csrc/config/sim_options.cc",
    "csrc/config/icnt_config.cc",
    "csrc/trace/trace.cc",
    "csrc/engine/cpu_engine.cc",
    "csrc/engine/check_engine.cc",
    "csrc/power/power.cc",
    "csrc/power/arch_energy.cc",
    "csrc/driver/simulator.cc",
    "csrc/driver/dump.cc",
    "csrc/driver/debugger.cc",
    "csrc/driver/icnt_bench.cc",
    "csrc/parallel/linksim.cc",
]
HIP_SRC = ["csrc/engine/gpu_engine.hip", "csrc/engine/engine_k_lds.hip", "csrc/engine/engine_k_prof.hip",
           "csrc/engine/engine_k_global.hip", "csrc/engine/engine_k_split.hip", "csrc/engine/engine_k_split2.hip", "csrc/engine/ingest_mfma.hip"]
STUB_SRC = ["csrc/engine/gpu_stub.cc"]


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def have_hipcc():
    return shutil.which("hipcc") is not None or os.path.exists(os.path.join(ROCM, "bin", "hipcc"))


def write_ninja(cpu_only: bool, extra_targets: bool) -> str:
    bdir = os.path.join(ROOT, "build")
    os.makedirs(bdir, exist_ok=True)
    hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    inc = " ".join(f"-I{p}" for p in [os.path.join(ROOT, "csrc")] + _pybind_includes())
    cxxflags = f"-std=c++17 -O3 -g -fPIC -fopenmp -pthread -Wall -Wno-unused-variable -Wno-unused-function {inc}"
    hipflags = (f"-std=c++17 -O3 -fPIC --offload-arch={ARCH} -munsafe-fp-atomics "
                f"-I{os.path.join(ROOT, 'csrc')}")
    ldflags = f"-fopenmp -pthread -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib"
    lines = [
        "ninja_required_version = 1.3",
        f"cxxflags = {cxxflags}",
        f"hipflags = {hipflags}",
        f"ldflags = {ldflags}",
        "rule cxx",
        "  command = g++ $cxxflags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule hip",
        f"  command = {hipcc} $hipflags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        "rule link_so",
        "  command = g++ -shared $in -o $out $ldflags $libs",
        "  description = LINK $out",
        "rule link_exe",
        "  command = g++ $in -o $out $ldflags $libs",
        "  description = LINK $out",
        "rule hipexe",
        f"  command = {hipcc} $hipflags $in -o $out $libs",
        "rule isatrace",
        f"  command = {sys.executable} {os.path.join(PKG, 'isatrace', 'build.py')} $in -o $out \"--libs=$libs\" -- "
        f"-munsafe-fp-atomics -fPIC -I{os.path.join(ROOT, 'csrc')}",
        "  description = HIPEXE $out",
        # binary-only path: device code recovered from the precompiled app
        # (isatrace/binary.py), host half from the source
        "rule isatrace_bin",
        f"  command = {sys.executable} {os.path.join(PKG, 'isatrace', 'build.py')} $src -o $out --device-from $in "
        f"\"--libs=$libs\" -- -munsafe-fp-atomics -fPIC -I{os.path.join(ROOT, 'csrc')}",
        "  description = HIPEXE-BIN $out",
    ]
    objs = []
    for s in CORE_SRC:
        o = os.path.join(bdir, s.replace("/", "_") + ".o")
        lines.append(f"build {o}: cxx {os.path.join(ROOT, s)}")
        objs.append(o)
    gpu_objs = []
    if not cpu_only:
        for s in HIP_SRC:
            o = os.path.join(bdir, s.replace("/", "_") + ".o")
            lines.append(f"build {o}: hip {os.path.join(ROOT, s)}")
            gpu_objs.append(o)
        libs = "-lamdhip64"
    else:
        for s in STUB_SRC:
            o = os.path.join(bdir, s.replace("/", "_") + ".o")
            lines.append(f"build {o}: cxx {os.path.join(ROOT, s)}")
            gpu_objs.append(o)
        libs = ""
    bind_o = os.path.join(bdir, "bindings.o")
    lines.append(f"build {bind_o}: cxx {os.path.join(ROOT, 'csrc/bindings/py_asim.cc')}")
    main_o = os.path.join(bdir, "main.o")
    lines.append(f"build {main_o}: cxx {os.path.join(ROOT, 'csrc/driver/main.cc')}")
    so = os.path.join(PKG, "_asim" + ext_suffix())
    lines.append(f"build {so}: link_so {' '.join(objs + gpu_objs + [bind_o])}")
    lines.append(f"  libs = {libs}")
    exe = os.path.join(ROOT, "bin", "accel-sim.out")
    lines.append(f"build {exe}: link_exe {' '.join(objs + gpu_objs + [main_o])}")
    lines.append(f"  libs = {libs}")
    defaults = [so, exe]
    if extra_targets and not cpu_only:
        ub_dir = os.path.join(ROOT, "csrc", "ubench")
        if os.path.isdir(ub_dir):
            for fn in sorted(os.listdir(ub_dir)):
                if fn.endswith(".hip"):
                    out = os.path.join(ROOT, "bin", "ubench", fn[:-4])
                    src = os.path.join(ub_dir, fn)
                    lines.append(f"build {out}: hipexe {src} | {os.path.join(ub_dir, 'ubench.h')}")
                    first = open(src).readline()
                    if first.startswith("// UB_LIBS:"):
                        lines.append(f"  libs = {first.split(':', 1)[1].strip()}")
                    defaults.append(out)
        # plain HIP applications: bin/apps/<app> (HW timing / counters) and the
        # automatically instrumented twin bin/isatrace/<app> (+ .asimisa map)
        # built from the same source with the same device flags
        app_dir = os.path.join(ROOT, "csrc", "apps")
        if os.path.isdir(app_dir):
            hdr = os.path.join(app_dir, "app_common.h")
            isa_deps = " ".join(os.path.join(ROOT, p) for p in (
                "accel_sim_framework_distributed_amd/isatrace/rewrite.py",
                "accel_sim_framework_distributed_amd/isatrace/build.py", "csrc/tracer/isa_runtime.cc"))
            for fn in sorted(os.listdir(app_dir)):
                if fn.endswith(".hip"):
                    out = os.path.join(ROOT, "bin", "apps", fn[:-4])
                    first = open(os.path.join(app_dir, fn)).readline()
                    libs = first.split(':', 1)[1].strip() if first.startswith("// UB_LIBS:") else ""
                    lines.append(f"build {out}: hipexe {os.path.join(app_dir, fn)} | {hdr}")
                    lines.append(f"  libs = {libs}")
                    defaults.append(out)
                    tout = os.path.join(ROOT, "bin", "isatrace", fn[:-4])
                    lines.append(f"build {tout}: isatrace {os.path.join(app_dir, fn)} | {hdr} {isa_deps}")
                    lines.append(f"  libs = {libs}")
                    defaults.append(tout)
                    if fn[:-4] in BINARY_PATH_APPS:
                        bout = os.path.join(ROOT, "bin", "isatrace_bin", fn[:-4])
                        lines.append(f"build {bout}: isatrace_bin {out} | {os.path.join(app_dir, fn)} {hdr} {isa_deps} "
                                     f"{os.path.join(PKG, 'isatrace', 'binary.py')}")
                        lines.append(f"  src = {os.path.join(app_dir, fn)}")
                        lines.append(f"  libs = {libs}")
                        defaults.append(bout)
        # examples/<name>/main.hip -> bin/examples/<name>
        ex_dir = os.path.join(ROOT, "examples")
        if os.path.isdir(ex_dir):
            hdr = os.path.join(ROOT, "csrc", "apps", "app_common.h")
            for name in sorted(os.listdir(ex_dir)):
                src = os.path.join(ex_dir, name, "main.hip")
                if os.path.exists(src):
                    out = os.path.join(ROOT, "bin", "examples", name)
                    tout = os.path.join(ROOT, "bin", "isatrace", name)
                    first = open(src).readline()
                    libs = first.split(':', 1)[1].strip() if first.startswith("// UB_LIBS:") else ""
                    lines.append(f"build {out}: hipexe {src} | {hdr}")
                    lines.append(f"  libs = {libs}")
                    lines.append(f"build {tout}: isatrace {src} | {hdr} {isa_deps}")
                    lines.append(f"  libs = {libs}")
                    defaults += [out, tout]
        tracer = os.path.join(ROOT, "csrc", "tracer", "asim_tracer.cc")
        if os.path.exists(tracer) and os.path.isdir(os.path.join(ROCM, "include", "rocprofiler-sdk")):
            t_o = os.path.join(bdir, "tracer.o")
            lines.append(f"build {t_o}: hip {tracer}")
            t_so = os.path.join(ROOT, "bin", "libasim_tracer.so")
            lines.append(f"build {t_so}: link_so {t_o}")
            lines.append(f"  libs = -lrocprofiler-sdk -ldl")
            defaults.append(t_so)
    lines.append("default " + " ".join(defaults))
    path = os.path.join(bdir, "build.ninja")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def build_dist_ext(verbose: bool = False) -> str:
    """The native epoch loop of the packet collective (csrc/parallel/exchange.cc)
    as a torch C++ extension (it calls c10d::ProcessGroup), built in-tree:
    accel_sim_framework_distributed_amd/_asim_dist.so."""
    import torch
    from torch.utils.cpp_extension import load
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    bdir = os.path.join(ROOT, "build", "dist_ext")
    os.makedirs(bdir, exist_ok=True)
    # the device-resident epoch loop's kernels (csrc/parallel/linksim_dev.hip),
    # compiled by hipcc for gfx950 and linked into the extension
    dev_src = os.path.join(ROOT, "csrc", "parallel", "linksim_dev.hip")
    dev_obj = os.path.join(bdir, "linksim_dev.o")
    deps = [dev_src] + [os.path.join(ROOT, "csrc", "parallel", f) for f in ("linksim_dev.h", "linksim_core.h", "linksim.h")]
    if not os.path.exists(dev_obj) or os.path.getmtime(dev_obj) < max(os.path.getmtime(d) for d in deps):
        hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
        subprocess.check_call([hipcc, "-std=c++17", "-O2", "-fPIC", f"--offload-arch={ARCH}",
                               f"-I{os.path.join(ROOT, 'csrc')}", "-c", dev_src, "-o", dev_obj])
        # the extension's ninja file does not track a prebuilt object: relink
        for f in ("_asim_dist.so", "build.ninja", ".ninja_log"):
            if os.path.exists(os.path.join(bdir, f)):
                os.remove(os.path.join(bdir, f))
    load(name="_asim_dist", sources=[os.path.join(ROOT, "csrc", "parallel", "exchange.cc"),
                                      os.path.join(ROOT, "csrc", "parallel", "linksim.cc")],
         build_directory=bdir, extra_cflags=["-O2", f"-I{os.path.join(ROOT, 'csrc')}", "-D__HIP_PLATFORM_AMD__=1"],
         extra_include_paths=[os.path.join(ROCM, "include")], verbose=verbose,
         extra_ldflags=[dev_obj, f"-L{ROCM}/lib", "-lamdhip64", f"-L{torch_lib}", "-lc10_hip"],
         with_cuda=False, is_python_module=True)
    out = os.path.join(PKG, "_asim_dist.so")
    shutil.copy2(os.path.join(bdir, "_asim_dist.so"), out)
    return out


def build(cpu_only: bool = False, jobs: int | None = None, extra: bool = True, verbose: bool = False) -> None:
    if not cpu_only and not have_hipcc():
        print("[build_native] hipcc not found: building the CPU engine only", file=sys.stderr)
        cpu_only = True
    os.makedirs(os.path.join(ROOT, "bin", "ubench"), exist_ok=True)
    nf = write_ninja(cpu_only, extra)
    j = jobs or min(16, os.cpu_count() or 4)
    cmd = ["ninja", "-f", nf, f"-j{j}"]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True, cwd=ROOT)
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch is part of the image
        print("[build_native] torch not importable: skipping the _asim_dist extension", file=sys.stderr)
        return
    build_dist_ext(verbose)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-only", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip ubench / tracer targets")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    build(a.cpu_only, a.j, not a.no_extra, a.v)
