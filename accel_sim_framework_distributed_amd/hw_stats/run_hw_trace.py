#!/usr/bin/env python3
"""Capture traces of HIP applications on MI355X (reference
util/tracer_nvbit/run_hw_trace.py:51-121: per benchmark create
``<out>/<app>/<args>/traces``, run the app with the tracer injected,
post-process).

Plain HIP applications are traced through their automatically instrumented
twins (``bin/isatrace/<app>``, built by isatrace/build.py from the same
source), which write ``kernel-N.traceg`` + ``kernelslist.g`` when
``ASIM_TRACE_DIR`` is set; this driver runs them, then (``--binary``)
converts each text trace to the simulator's binary ``.asimk`` format and
rewrites the kernelslist -- the post-processing step.  ``-l`` injects the
rocprofiler-sdk tool (bin/libasim_tracer.so) to also record RCCL calls and
dispatch metadata of un-annotated kernels.

    run_hw_trace.py -B asim_hip_apps -o hw_run/traces/device-0
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import common  # noqa: E402
else:
    from ..job_launching import common


def to_binary(trace_dir: str) -> int:
    """Convert every kernel-N.traceg listed in kernelslist.g to .asimk."""
    from accel_sim_framework_distributed_amd import _native
    mod = _native.load()
    kl = os.path.join(trace_dir, "kernelslist.g")
    lines = open(kl).read().splitlines()
    out, n = [], 0
    for ln in lines:
        s = ln.strip()
        if s.startswith("kernel-") and s.endswith(".traceg"):
            dst = s[:-len(".traceg")] + ".asimk"
            mod.convert_trace(os.path.join(trace_dir, s), os.path.join(trace_dir, dst))
            os.remove(os.path.join(trace_dir, s))
            out.append(dst)
            n += 1
        else:
            out.append(ln)
    with open(kl, "w") as f:
        f.write("\n".join(out) + "\n")
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-B", "--benchmark_list", required=True)
    ap.add_argument("-o", "--out", default=os.path.join(common.REPO_ROOT, "hw_run", "traces", "device-0"))
    ap.add_argument("-b", "--binary", action="store_true", help="convert traces to .asimk")
    ap.add_argument("-l", "--rocprof_tool", action="store_true", help="also inject bin/libasim_tracer.so")
    ap.add_argument("-t", "--timeout", type=int, default=600)
    ap.add_argument("-n", "--dry_run", action="store_true")
    ap.add_argument("--no_isa", dest="isa", action="store_false",
                    help="run bin/apps/<app> itself instead of its isatrace twin bin/isatrace/<app>")
    o = ap.parse_args(argv)
    reg = common.Registry()
    for exec_dir, data_dir, app, args_list in reg.benchmarks(o.benchmark_list.split(",")):
        exe_path = os.path.join(os.path.expandvars(exec_dir) or ".", app)
        if not os.path.isabs(exe_path):
            exe_path = os.path.join(common.REPO_ROOT, exe_path)
        # the automatically instrumented twin of a plain HIP app (isatrace)
        twin = os.path.join(common.REPO_ROOT, "bin", "isatrace", app)
        if o.isa and os.path.exists(twin) and os.path.exists(twin + ".asimisa"):
            exe_path = twin
        for a in args_list:
            args = a.get("args")
            tdir = os.path.abspath(os.path.join(o.out, app, common.argfoldername(args), "traces"))
            env = dict(os.environ, ASIM_TRACE_DIR=tdir)
            if o.rocprof_tool:
                env["ROCP_TOOL_LIBRARIES"] = os.path.join(common.REPO_ROOT, "bin", "libasim_tracer.so")
            cmd = ["timeout", "-k", "10", str(o.timeout), exe_path] + (shlex.split(str(args)) if args else [])
            print(f"ASIM_TRACE_DIR={tdir} " + " ".join(shlex.quote(c) for c in cmd), flush=True)
            if o.dry_run:
                continue
            os.makedirs(tdir, exist_ok=True)
            rc = subprocess.call(cmd, env=env)
            if rc != 0:
                print(f"run_hw_trace: {app} failed (rc={rc}); stopping", file=sys.stderr)
                return rc
            if o.binary:
                print(f"  converted {to_binary(tdir)} kernels to .asimk")
    return 0


if __name__ == "__main__":
    sys.exit(main())
