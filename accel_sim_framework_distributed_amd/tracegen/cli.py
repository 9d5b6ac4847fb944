#!/usr/bin/env python3
"""Trace utilities (the reference's util/tracer_nvbit helpers and others/ tools):

  generate   synthetic Rodinia-2.0-ft-shaped traces in the downloaded-trace
             layout (stands in for get-accel-sim-traces.py:67-172: no network)
  convert    .traceg <-> .asimk for a trace directory (post-processing step,
             reference post-traces-processing.cpp)
  info       per-kernel stats.csv of a trace directory (tracer stats.csv)
  occupancy  CTAs per SM and the limiting resource for each kernel under a
             config (others/occupancy_calc_tool)
  bbv        per-kernel basic-block vectors (others/bbv_tool): execution
             counts of each basic block (PC ranges split at branches/barriers),
             weighted by active threads, for sampling / SimPoint selection
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import Counter
from typing import Dict, List

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd import _native  # noqa: E402
    from accel_sim_framework_distributed_amd.tracegen import format as tfmt, rodinia  # noqa: E402
else:
    from .. import _native
    from . import format as tfmt, rodinia


def kernel_files(trace_dir: str) -> List[str]:
    kl = os.path.join(trace_dir, "kernelslist.g")
    out = []
    for line in open(kl):
        s = line.strip()
        if s.startswith("kernel-"):
            out.append(os.path.join(trace_dir, s))
    return out


def cmd_generate(a) -> int:
    out = os.path.join(a.out, a.device, "rodinia_2.0-ft")
    res = rodinia.generate_suite(out, a.apps.split(",") if a.apps else None, text=a.text)
    for app, kl in res.items():
        print(f"{app}: {kl}")
    return 0


def cmd_convert(a) -> int:
    mod = _native.load()
    kl = os.path.join(a.dir, "kernelslist.g")
    lines = open(kl).read().splitlines()
    out = []
    for ln in lines:
        s = ln.strip()
        if a.to == "binary" and s.endswith(".traceg"):
            dst = s[:-len(".traceg")] + ".asimk"
            mod.convert_trace(os.path.join(a.dir, s), os.path.join(a.dir, dst))
            out.append(dst)
        elif a.to == "text" and s.endswith(".asimk"):
            dst = s[:-len(".asimk")] + ".traceg"
            tfmt.write_kernel_text(os.path.join(a.dir, dst), tfmt.read_kernel_binary(os.path.join(a.dir, s)))
            out.append(dst)
        else:
            out.append(ln)
    if not a.keep:
        for ln, new in zip(lines, out):
            if ln.strip() != new.strip():
                os.remove(os.path.join(a.dir, ln.strip()))
    with open(kl, "w") as f:
        f.write("\n".join(out) + "\n")
    print(f"converted {sum(1 for x, y in zip(lines, out) if x.strip() != y.strip())} kernels in {a.dir}")
    return 0


def cmd_info(a) -> int:
    mod = _native.load()
    print("kernel id, kernel name, grid_dim, block_dim, #warp insts, #thread insts")
    for p in kernel_files(a.dir):
        k = mod.kernel_info(p)
        g, b = tuple(k["grid"]), tuple(k["block"])
        print(f"{os.path.basename(p).split('.')[0]}, {k['name']}, {g}, {b}, {k['warp_insts']}, {k['thread_insts']}")
    return 0


def cmd_occupancy(a) -> int:
    from ..models import presets
    mod = _native.load()
    args = presets.args_for(a.config) if not a.config_file else ["-config", a.config_file]
    for p in kernel_files(a.dir):
        k = mod.kernel_info(p)
        threads = k["block"][0] * k["block"][1] * k["block"][2]
        o = mod.occupancy(args, threads, k["shmem"], k["nregs"])
        print(f"{os.path.basename(p)} {k['name']}: {o['cta_per_sm']} CTAs/SM, limited by {o['limiter']}")
    return 0


def basic_block_vector(k: tfmt.KernelArrays) -> Dict[int, int]:
    """{block start PC: thread-weighted executions}; a block ends after a
    branch, barrier or exit, or where another stream's PC sequence enters."""
    names = k.opnames
    ins = k.insts
    enders = set()
    for i, n in enumerate(names):
        u = n.upper()
        if any(t in u for t in ("BRA", "BRANCH", "BAR", "EXIT", "ENDPGM", "JMP", "RET", "CALL")):
            enders.add(i)
    # leaders: first PC of every stream and every PC following a block ender
    leaders = set()
    for s in k.streams:
        b, c = int(s["begin"]), int(s["count"])
        if c:
            leaders.add(int(ins["pc"][b]))
        for j in range(b, b + c - 1):
            if int(ins["opcode"][j]) in enders:
                leaders.add(int(ins["pc"][j + 1]))
    bbv: Counter = Counter()
    masks = ins["mask"]
    for s in k.streams:
        b, c = int(s["begin"]), int(s["count"])
        cur = None
        for j in range(b, b + c):
            pc = int(ins["pc"][j])
            if pc in leaders or cur is None:
                cur = pc
            bbv[cur] += bin(int(masks[j])).count("1")
    return dict(sorted(bbv.items()))


def cmd_bbv(a) -> int:
    res = {}
    for p in kernel_files(a.dir):
        if not p.endswith(".asimk"):
            print(f"bbv: {p} is not binary; run `convert --to binary` first", file=sys.stderr)
            return 1
        k = tfmt.read_kernel_binary(p)
        res[os.path.basename(p)] = {hex(pc): n for pc, n in basic_block_vector(k).items()}
    text = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(text)
    else:
        print(text)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    g = sub.add_parser("generate")
    g.add_argument("-o", "--out", default="hw_run/traces")
    g.add_argument("-d", "--device", default="synthetic-QV100")
    g.add_argument("-a", "--apps", default="")
    g.add_argument("--text", action="store_true")
    c = sub.add_parser("convert")
    c.add_argument("dir")
    c.add_argument("--to", choices=["binary", "text"], default="binary")
    c.add_argument("--keep", action="store_true", help="keep the source files")
    i = sub.add_parser("info")
    i.add_argument("dir")
    o = sub.add_parser("occupancy")
    o.add_argument("dir")
    o.add_argument("-C", "--config", default="QV100")
    o.add_argument("--config_file", default="")
    b = sub.add_parser("bbv")
    b.add_argument("dir")
    b.add_argument("-o", "--out", default="")
    a = ap.parse_args(argv)
    return {"generate": cmd_generate, "convert": cmd_convert, "info": cmd_info, "occupancy": cmd_occupancy,
            "bbv": cmd_bbv}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
