#!/usr/bin/env python3
"""Launch a grid of simulations: every (benchmark, args) x config.

Same CLI and run-directory layout as the reference
(util/job_launching/run_simulations.py + common.py:175-217):

    run_simulations.py -B rodinia_2.0-ft -C QV100-SASS -T <trace_root> -N myrun

creates ``<run_dir>/<app>/<argfolder>/<config>/`` with ``gpgpusim.config``
(base + extras + trace.config), a ``traces`` symlink, ``justrun.sh`` and the
job script, submits the job to slurm (``sbatch``), torque (``qsub``) or the
local manager (``procman.py``), and appends one line per job to
``logfiles/sim_log.<name>.<date>.txt`` (read by job_status / get_stats /
monitor_func_test).  The simulator is this framework's native
``bin/accel-sim.out``; ``-C X-GPU`` selects the MI355X cycle engine and
procman then hands each job a GPU slot.
"""
from __future__ import annotations

import argparse
import datetime
import glob
import os
import shutil
import subprocess
import sys
from typing import List, Optional

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import common  # noqa: E402
else:
    from . import common


def find_traces(trace_dir: str, app: str, argfolder: str) -> Optional[str]:
    sub = os.path.join(app, argfolder)
    tries = [os.path.join(trace_dir, sub, "traces")]
    tries += glob.glob(os.path.join(trace_dir, "*", "*", sub, "traces"))
    tries += glob.glob(os.path.join(trace_dir, "*", sub, "traces"))
    for t in tries:
        if os.path.isdir(t):
            return os.path.abspath(t)
    return None


def pick_launcher(name: str):
    """(submit command list, kind)."""
    procman = [sys.executable, os.path.join(common.HERE, "procman.py")]
    if name in ("sbatch", "slurm"):
        return ["sbatch"], "slurm"
    if name in ("qsub", "torque"):
        return ["qsub"], "torque"
    if name in ("local", "procman"):
        return procman, "procman"
    if name == "":
        if shutil.which("sbatch"):
            return ["sbatch"], "slurm"
        if shutil.which("qsub"):
            return ["qsub"], "torque"
        print("Cannot find a supported job management system. Spawning jobs locally.")
        return procman, "procman"
    raise SystemExit(f"unknown launcher {name!r} (sbatch | qsub | local)")


def job_id_from(out: str, kind: str) -> str:
    toks = out.strip().split()
    if not toks:
        raise RuntimeError("job submission printed no job id")
    if kind == "slurm":
        return toks[-1]          # "Submitted batch job 123"
    if kind == "torque":
        return toks[0].split(".")[0]
    return toks[0]


def setup_run(o, reg: common.Registry, cfg_name: str, extra: str, base_cfg: str, exec_dir: str, data_dir: str,
              app: str, arg: dict, version: str, sim_bin: str, launcher, kind: str, log_lines: List[str]) -> None:
    args = arg.get("args")
    argfolder = common.argfoldername(args)
    run_dir = os.path.join(o.run_directory, app.replace("/", "_"), argfolder, cfg_name)
    os.makedirs(run_dir, exist_ok=True)
    if o.trace_dir:
        tdir = find_traces(o.trace_dir, app, argfolder)
        if tdir is None:
            raise SystemExit(f"Cannot find traces for {app}/{argfolder} under {o.trace_dir}")
        link = os.path.join(run_dir, "traces")
        if os.path.lexists(link):
            os.remove(link)
        os.symlink(tdir, link)
    # gpgpusim.config = base + app-specific + extras (+ trace.config)
    text = open(base_cfg).read()
    app_opts = os.path.expandvars(os.path.join("$GPUAPPS_ROOT", "benchmarks", "app-specific-gpgpu-sim-options", app,
                                               "benchmark_options.txt"))
    if os.path.isfile(app_opts):
        text += "\n" + open(app_opts).read().strip() + "\n"
    text += "\n" + extra + "\n"
    if o.accelwattch_HW:
        text += f"\n-hw_perf_bench_name {app}\n"
    tcfg = os.path.join(os.path.dirname(base_cfg), "trace.config")
    if o.trace_dir and os.path.exists(tcfg):
        text += "\n# Accel-Sim Parameters\n" + open(tcfg).read()
    with open(os.path.join(run_dir, "gpgpusim.config"), "w") as f:
        f.write(text)
    # side files the config refers to by relative name (power XMLs, icnt, hw csv)
    for side in glob.glob(os.path.join(os.path.dirname(base_cfg), "*")):
        if side.endswith((".xml", ".icnt", ".csv")):
            shutil.copy2(side, run_dir)

    if o.trace_dir:
        command = f"{sim_bin} -config ./gpgpusim.config -trace ./traces/kernelslist.g"
    else:
        command = os.path.join(os.path.expandvars(exec_dir), app) + ("" if args is None else " " + str(args))
    name = f"{app}-{argfolder}.{version}"
    mem = o.job_mem or arg.get("accel-sim-mem", "4G")
    tmpl = open(os.path.join(common.HERE, "templates", "job.sim")).read()
    rep = {"NAME": name, "SUBDIR": run_dir, "MEM_USAGE": mem, "COMMAND": command,
           "PREFIX": o.benchmark_exec_prefix, "THREADS": str(o.threads)}
    for k, v in rep.items():
        tmpl = tmpl.replace("REPLACE_" + k, v)
    script = os.path.join(run_dir, "job.sim")
    with open(script, "w") as f:
        f.write(tmpl)
    justrun = os.path.join(run_dir, "justrun.sh")
    with open(justrun, "w") as f:
        f.write(f"#!/bin/bash\ncd {run_dir}\n{o.benchmark_exec_prefix} {command}\n")
    os.chmod(justrun, 0o755)
    if o.no_launch:
        return
    cmd = launcher + [script]
    r = subprocess.run(cmd, cwd=run_dir, capture_output=True, text=True)
    if r.returncode != 0:
        print(f"job submission failed for {run_dir}:\n{r.stdout}{r.stderr}")
        return
    jid = job_id_from(r.stdout, kind)
    stamp = datetime.datetime.now().strftime("%H:%M:%S")
    log_lines.append(f"{stamp}\t{jid}\t{app}\t{argfolder}\t{cfg_name}\t{name}")
    print(f"Job {jid} submitted: {app} {argfolder} {cfg_name}")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-B", "--benchmark_list", default="", help="comma separated suites (apps/define-*.yml)")
    ap.add_argument("-C", "--configs_list", default="", help="comma separated BASE-EXTRA... configs")
    ap.add_argument("-p", "--benchmark_exec_prefix", default="", help="prefix of the simulator command (e.g. gdb)")
    ap.add_argument("-r", "--run_directory", default="", help="root of the run directories")
    ap.add_argument("-n", "--no_launch", action="store_true", help="set up run directories only")
    ap.add_argument("-s", "--simulator_dir", default="", help="directory holding accel-sim.out")
    ap.add_argument("-N", "--launch_name", default="", help="name of the launch (logfile name)")
    ap.add_argument("-T", "--trace_dir", default="", help="trace root: trace-driven mode")
    ap.add_argument("-M", "--job_mem", default=None, help="job memory request, e.g. 4G")
    ap.add_argument("-l", "--launcher", default="", help="sbatch | qsub | local")
    ap.add_argument("-c", "--cores", default=None, help="procman core limit")
    ap.add_argument("-g", "--gpus", type=int, default=None, help="procman GPU slots (GPU engine jobs)")
    ap.add_argument("-a", "--accelwattch_HW", action="store_true", help="pass -hw_perf_bench_name <app>")
    ap.add_argument("--threads", type=int, default=1, help="OpenMP threads per CPU-engine job")
    o = ap.parse_args(argv)
    if not o.benchmark_list or not o.configs_list:
        ap.error("-B and -C are required")
    return o


def main(argv=None) -> int:
    o = parse(argv)
    reg = common.Registry()
    if o.run_directory == "":
        o.run_directory = os.path.join(common.REPO_ROOT, "sim_run")
    o.run_directory = os.path.abspath(o.run_directory)
    if o.trace_dir:
        o.trace_dir = os.path.abspath(os.path.expandvars(o.trace_dir))
    version = common.build_version()
    # a private copy of the simulator per build version (reference
    # gpgpu-sim-builds/<version>) so rebuilding does not disturb running jobs
    src_bin = os.path.join(o.simulator_dir, "accel-sim.out") if o.simulator_dir else common.simulator_binary()
    bdir = os.path.join(o.run_directory, "gpgpu-sim-builds", version)
    os.makedirs(bdir, exist_ok=True)
    sim_bin = os.path.join(bdir, "accel-sim.out")
    if not os.path.exists(sim_bin) or os.path.getmtime(sim_bin) < os.path.getmtime(src_bin):
        shutil.copy2(src_bin, sim_bin)
    launcher, kind = pick_launcher(o.launcher)
    benches = reg.benchmarks([b for b in o.benchmark_list.split(",") if b])
    cfgs = [reg.config(c) for c in o.configs_list.split(",") if c]
    print(f"Running simulations with {version}\nUsing configs: {o.configs_list}\nBenchmark: {o.benchmark_list}")
    log_lines: List[str] = []
    for cfg_name, extra, base_cfg in cfgs:
        for exec_dir, data_dir, app, args_list in benches:
            for arg in args_list:
                setup_run(o, reg, cfg_name, extra, base_cfg, exec_dir, data_dir, app, arg, version, sim_bin,
                          launcher, kind, log_lines)
    if log_lines:
        now = datetime.datetime.now()
        tag = (o.launch_name + ".") if o.launch_name else ""
        path = os.path.join(common.log_dir(), f"sim_log.{tag}{now.strftime('%y.%m.%d-%H:%M:%S')}.txt")
        with open(path, "a") as f:
            f.write("\n".join(log_lines) + "\n")
        print(f"Launch log: {path}")
    if kind == "procman" and not o.no_launch:
        cmd = launcher + ["-S"]
        if o.cores:
            cmd += ["-c", str(o.cores)]
        if o.gpus is not None:
            cmd += ["-g", str(o.gpus)]
        subprocess.call(cmd)
    return 0


if __name__ == "__main__":
    sys.exit(main())
