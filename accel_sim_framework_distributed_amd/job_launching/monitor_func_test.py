#!/usr/bin/env python3
"""Wait for a launch to finish and fail if any job failed
(reference util/job_launching/monitor_func_test.py:72-97).

Polls job_status every ``-S`` seconds until every job left the queue, then
prints the status table, optionally collects stats into ``-s <csv>`` via
get_stats, and exits non-zero if a job failed (unless ``-I``).  ``-T`` bounds
the wait; with ``-K`` the remaining jobs are killed when it expires.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import common, get_stats, job_status, procman  # noqa
else:
    from . import common, get_stats, job_status, procman


def kill_jobs(infos, mgr: str) -> None:
    import subprocess
    for j in infos:
        if j["status"] not in job_status.UNFINISHED:
            continue
        if mgr == "squeue":
            subprocess.call(["scancel", j["jobid"]])
        elif mgr == "qstat":
            subprocess.call(["qdel", j["jobid"]])
    if mgr == "procman":
        procman.kill_all(procman.default_state_file())


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-l", "--logfile", default="")
    ap.add_argument("-r", "--run_dir", default="")
    ap.add_argument("-N", "--sim_name", default="")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-s", "--statsfile", default="", help="write get_stats CSV here when done")
    ap.add_argument("-S", "--sleep_time", type=float, default=30)
    ap.add_argument("-I", "--ignore_failures", action="store_true")
    ap.add_argument("-T", "--timeout", type=float, default=99999)
    ap.add_argument("-K", "--killwhentimedout", action="store_true")
    ap.add_argument("-j", "--job_manager", default=None)
    o = ap.parse_args(argv)
    run_dir = os.path.abspath(o.run_dir) if o.run_dir else os.path.join(common.REPO_ROOT, "sim_run")
    mgr = job_status.detect_manager(o.job_manager)
    log = job_status.logfiles(o.logfile, o.sim_name)[0]
    t0 = time.time()
    while True:
        infos = job_status.job_infos(log, run_dir, mgr)
        pending = [j for j in infos if j["status"] in job_status.UNFINISHED]
        if o.verbose:
            print(job_status.print_table(infos))
        else:
            print(f"[{time.time() - t0:7.0f}s] {len(infos) - len(pending)}/{len(infos)} jobs finished", flush=True)
        if not pending:
            break
        if time.time() - t0 > o.timeout:
            print(f"timed out after {o.timeout}s with {len(pending)} jobs unfinished")
            if o.killwhentimedout:
                kill_jobs(infos, mgr)
            print(job_status.print_table(infos))
            return 1
        time.sleep(o.sleep_time)
    print(job_status.print_table(infos))
    failed = [j for j in infos if j["status"] not in job_status.PASSING]
    if o.statsfile:
        csv = get_stats.collect(log, run_dir, get_stats.load_stats_yml(""), per_kernel=False)
        with open(o.statsfile, "w") as f:
            f.write(get_stats.render_csv(csv, configs_as_rows=False))
        print(f"stats written to {o.statsfile}")
    if failed and not o.ignore_failures:
        print(f"{len(failed)} jobs failed")
        return 1
    print("Congratulations! All jobs passed!" if not failed else f"{len(failed)} failures ignored")
    return 0


if __name__ == "__main__":
    sys.exit(main())
