#!/usr/bin/env python3
"""Status table of the jobs of a launch (reference util/job_launching/job_status.py).

Reads a ``logfiles/sim_log.*`` file written by run_simulations.py, asks the job
manager (procman / squeue / qstat) whether each job is still queued or
running, classifies finished jobs from their output (exit detected, deadlock,
assertion, segfault, ...) and prints a table with the basic simulator stats.
``job_infos()`` is the programmatic entry point used by monitor_func_test.py.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import shutil
import subprocess
import sys
from typing import Dict, List, Optional

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import common, procman  # noqa: E402
else:
    from . import common, procman

# searched in stdout/stderr of finished jobs, first match wins
FAILURE_PATTERNS = [
    (r"deadlock detected", "DEADLOCK"),
    (r"Assertion", "ASSERT"),
    (r"Segmentation fault", "SEGF"),
    (r"Aborted", "ABORTED"),
    (r"GPGPU-Sim \*\* ERROR", "SIM_ERROR"),
    (r"out of memory|MemoryError", "OOM"),
    (r"PBS: job killed|DUE TO TIME LIMIT|CANCELLED", "KILLED"),
    (r"FAILED|Failed|failed", "FUNC_TEST_FAILED"),
]
PASS_PATTERNS = [(r"PASSED|passed", "FUNC_TEST_PASSED")]

STATS_TO_PULL = {
    "SIM_TIME": r"gpgpu_simulation_time\s*=[^1-9]*(.*)",
    "TOT_INSN": r"gpu_tot_sim_insn\s*=\s*(.*)",
    "TOT_IPC": r"gpu_tot_ipc\s*=\s*(.*)",
    "TOT_CYCLE": r"gpu_tot_sim_cycle\s*=\s*(.*)",
    "SIMRATE_IPS": r"gpgpu_simulation_rate\s*=\s*(.*)\s*\(inst/sec\)",
}


def logfiles(logfile: str = "", sim_name: str = "") -> List[str]:
    d = common.log_dir()
    if logfile and logfile != "all":
        return [common.file_or_rel(logfile)]
    logs = glob.glob(os.path.join(d, "sim_log.*"))
    if sim_name:
        logs = [l for l in logs if os.path.basename(l).startswith(f"sim_log.{sim_name}.")]
    if not logs:
        raise SystemExit(f"no launch logs in {d}" + (f" for -N {sim_name}" if sim_name else ""))
    return sorted(logs, key=os.path.getmtime) if logfile == "all" else [max(logs, key=os.path.getmtime)]


def parse_log(path: str) -> List[Dict]:
    jobs = []
    for line in open(path):
        f = line.split()
        if len(f) != 6:
            continue
        jobs.append(dict(time=f[0], jobid=f[1], app=f[2], args=f[3], config=f[4], name=f[5]))
    return jobs


def detect_manager(name: Optional[str]) -> str:
    if name:
        return {"slurm": "squeue", "sbatch": "squeue", "torque": "qstat", "qsub": "qstat",
                "local": "procman"}.get(name, name)
    if shutil.which("squeue"):
        return "squeue"
    if shutil.which("qstat"):
        return "qstat"
    return "procman"


def manager_state(mgr: str, jobid: str) -> str:
    """QUEUED / RUNNING / FINISHED (manager no longer tracks it) / FAILED / KILLED."""
    if mgr == "procman":
        j = procman.job_state(procman.default_state_file(), int(jobid)) if jobid.isdigit() else None
        if j is None:
            return "FINISHED"
        if j["state"] == procman.RUNNING and not procman.pid_alive(j["pid"]):
            return "FINISHED"
        return {procman.QUEUED: "QUEUED", procman.RUNNING: "RUNNING", procman.KILLED: "KILLED"}.get(j["state"],
                                                                                                   "FINISHED")
    try:
        if mgr == "squeue":
            out = subprocess.run(["squeue", "-h", "-j", jobid, "-o", "%T"], capture_output=True, text=True,
                                 timeout=30).stdout.strip()
            return {"PENDING": "QUEUED", "RUNNING": "RUNNING", "COMPLETING": "RUNNING"}.get(out, "FINISHED")
        out = subprocess.run(["qstat", jobid], capture_output=True, text=True, timeout=30).stdout
        m = re.search(rf"^{re.escape(jobid)}\S*\s+\S+\s+\S+\s+\S+\s+(\w)", out, re.M)
        return {"Q": "QUEUED", "R": "RUNNING", "H": "QUEUED"}.get(m.group(1) if m else "", "FINISHED")
    except (OSError, subprocess.TimeoutExpired):
        return "FINISHED"


def classify(out_text: str, err_text: str) -> str:
    both = out_text + "\n" + err_text
    for pat, st in FAILURE_PATTERNS:
        if re.search(pat, both):
            return st
    if "*** exit detected ***" in out_text:
        for pat, st in PASS_PATTERNS:
            if re.search(pat, out_text):
                return st
        return "COMPLETE_NO_OTHER_INFO"
    return "NO_EXIT_DETECTED"


def pull_stats(text: str) -> Dict[str, str]:
    out = {}
    for k, pat in STATS_TO_PULL.items():
        ms = re.findall(pat, text)
        if ms:
            out[k] = ms[-1].strip()
    return out


def job_infos(log: str, run_dir: str, mgr: str) -> List[Dict]:
    res = []
    for j in parse_log(log):
        d = os.path.join(run_dir, j["app"].replace("/", "_"), j["args"], j["config"])
        outf = os.path.join(d, f"{j['name']}.o{j['jobid']}")
        errf = os.path.join(d, f"{j['name']}.e{j['jobid']}")
        out_text = open(outf, errors="replace").read() if os.path.exists(outf) else ""
        err_text = open(errf, errors="replace").read() if os.path.exists(errf) else ""
        ms = manager_state(mgr, j["jobid"])
        if ms in ("QUEUED", "RUNNING"):
            status = "WAITING_TO_RUN" if ms == "QUEUED" else "RUNNING"
        elif ms == "KILLED":
            status = "KILLED"
        else:
            status = classify(out_text, err_text)
        j.update(status=status, outfile=outf, errfile=errf, run_dir=d, stats=pull_stats(out_text),
                 out_tail=out_text.splitlines()[-10:], err_tail=err_text.splitlines()[-10:])
        res.append(j)
    return res


PASSING = ("COMPLETE_NO_OTHER_INFO", "FUNC_TEST_PASSED")
UNFINISHED = ("WAITING_TO_RUN", "RUNNING")


def print_table(infos: List[Dict], num_lines: int = 10) -> str:
    row = "{:<10.10} {:<34.34} {:<24.24} {:<18.18} {:<24.24} {}"
    lines = [row.format("job", "app", "args", "config", "status", "stats"), "-" * 150]
    fails = []
    for j in infos:
        stats = " ".join(f"{k}={v}" for k, v in j["stats"].items())
        lines.append(row.format(j["jobid"], j["app"], j["args"], j["config"], j["status"], stats))
        if j["status"] not in PASSING + UNFINISHED:
            fails.append(j)
    n_pass = sum(j["status"] in PASSING for j in infos)
    n_run = sum(j["status"] in UNFINISHED for j in infos)
    lines.append(f"\n{n_pass}/{len(infos)} passed, {n_run} still running or queued, {len(fails)} failed")
    for j in fails:
        lines.append(f"\n---- {j['app']} {j['args']} {j['config']}: {j['status']} ({j['outfile']})")
        lines += j["out_tail"][-num_lines:] + j["err_tail"][-num_lines:]
    return "\n".join(lines)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-l", "--logfile", default="", help="launch log (default: latest; 'all' = every log)")
    ap.add_argument("-n", "--num_lines", type=int, default=10, help="output lines shown for failed jobs")
    ap.add_argument("-r", "--run_dir", default="", help="run directory root")
    ap.add_argument("-j", "--job_manager", default=None, help="procman | squeue | qstat")
    ap.add_argument("-N", "--sim_name", default="", help="status of the latest launch with this -N name")
    o = ap.parse_args(argv)
    run_dir = os.path.abspath(o.run_dir) if o.run_dir else os.path.join(common.REPO_ROOT, "sim_run")
    mgr = detect_manager(o.job_manager)
    for log in logfiles(o.logfile, o.sim_name):
        print(f"Using logfile {log}")
        print(print_table(job_infos(log, run_dir, mgr), o.num_lines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
