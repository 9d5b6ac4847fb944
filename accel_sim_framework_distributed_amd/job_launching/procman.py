#!/usr/bin/env python3
"""Local job manager (the framework's stand-in for slurm/torque).

Behaviour of the reference's util/job_launching/procman.py:392-420 (queue
scripts, start a detached manager that runs them with bounded concurrency,
print state, kill, self-test, look a job up by id) with a different design:
the queue is a JSON file guarded by an ``fcntl`` lock instead of a pickled
object, and the manager is one detached process that hands out *device
slots* -- each job gets ``HIP_VISIBLE_DEVICES`` / ``ASIM_SLOT`` so GPU-engine
simulations spread over the node's MI355X GPUs (several per GPU: a QV100
simulation needs 112 of 256 CUs, see parallel/multi_gpu.py).

Usage::

    procman.py job1.sh job2.sh     # queue (prints job ids)
    procman.py -S [-c CORES] [-g GPUS] [--per-gpu K]   # start manager
    procman.py -p                  # print state
    procman.py -j ID               # state of one job
    procman.py -w                  # wait until the queue is empty
    procman.py -k                  # kill running jobs, clear the queue
    procman.py -s                  # self test
"""
from __future__ import annotations

import argparse
import fcntl
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
from contextlib import contextmanager
from typing import Dict, List, Optional

QUEUED, RUNNING, DONE, FAILED, KILLED = "QUEUED", "RUNNING", "COMPLETE", "FAILED", "KILLED"


def default_state_file() -> str:
    return os.environ.get("PROCMAN_STATE", os.path.join(tempfile.gettempdir(), f"asim_procman_{os.getuid()}.json"))


@contextmanager
def locked_state(path: str):
    """Read-modify-write the state file under an exclusive lock."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path + ".lock", "a+") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            st = json.load(open(path)) if os.path.exists(path) and os.path.getsize(path) else {}
        except json.JSONDecodeError:
            st = {}
        st.setdefault("next_id", 1)
        st.setdefault("jobs", {})
        st.setdefault("manager_pid", 0)
        yield st
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f, indent=1)
        os.replace(tmp, path)
        fcntl.flock(lk, fcntl.LOCK_UN)


def read_state(path: str) -> Dict:
    with locked_state(path) as st:
        return json.loads(json.dumps(st))


def pid_alive(pid: int) -> bool:
    if pid <= 0:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    # zombie children of the manager count as dead
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except OSError:
        return True


def submit(path: str, scripts: List[str], cwd: Optional[str] = None) -> List[int]:
    ids = []
    with locked_state(path) as st:
        for s in scripts:
            jid = st["next_id"]
            st["next_id"] += 1
            st["jobs"][str(jid)] = dict(script=os.path.abspath(s), cwd=cwd or os.path.dirname(os.path.abspath(s)),
                                        state=QUEUED, pid=0, rc=None, slot=None, submitted=time.time(),
                                        started=None, ended=None)
            ids.append(jid)
    return ids


def _slots(cores: int, gpus: int, per_gpu: int) -> List[Dict]:
    if gpus > 0:
        return [dict(gpu=g, k=k) for k in range(per_gpu) for g in range(gpus)]
    return [dict(gpu=None, k=k) for k in range(max(1, cores))]


def manager_loop(path: str, cores: int, gpus: int, per_gpu: int, sleep: float) -> None:
    """Run queued jobs until none is left (the detached manager process)."""
    slots = _slots(cores, gpus, per_gpu)
    busy: Dict[int, subprocess.Popen] = {}   # slot index -> process
    owner: Dict[int, str] = {}               # slot index -> job id
    idle_since = None
    while True:
        with locked_state(path) as st:
            if st["manager_pid"] != os.getpid():
                # killed / superseded
                for p in busy.values():
                    _kill_group(p.pid)
                return
            for si, p in list(busy.items()):
                rc = p.poll()
                if rc is None:
                    continue
                job = st["jobs"].get(owner[si])
                if job is not None and job["state"] == RUNNING:
                    job["state"] = DONE if rc == 0 else FAILED
                    job["rc"] = rc
                    job["ended"] = time.time()
                del busy[si], owner[si]
            queued = sorted((int(k) for k, j in st["jobs"].items() if j["state"] == QUEUED))
            for si in range(len(slots)):
                if not queued:
                    break
                if si in busy:
                    continue
                jid = str(queued.pop(0))
                job = st["jobs"][jid]
                env = dict(os.environ)
                env["PROCMAN_JOB_ID"] = jid
                env["ASIM_SLOT"] = str(si)
                if slots[si]["gpu"] is not None:
                    env["HIP_VISIBLE_DEVICES"] = str(slots[si]["gpu"])
                log = open(os.path.join(job["cwd"], f".procman.{jid}.log"), "w")
                p = subprocess.Popen(["bash", job["script"]], cwd=job["cwd"], env=env, stdout=log,
                                     stderr=subprocess.STDOUT, start_new_session=True)
                log.close()
                busy[si], owner[si] = p, jid
                job.update(state=RUNNING, pid=p.pid, slot=si, started=time.time())
            active = busy or any(j["state"] == QUEUED for j in st["jobs"].values())
            if not active:
                idle_since = idle_since or time.time()
                if time.time() - idle_since > 2 * sleep:
                    st["manager_pid"] = 0
                    return
            else:
                idle_since = None
        time.sleep(sleep)


def _kill_group(pid: int) -> None:
    # every job runs in its own session: its process group id is its pid
    try:
        os.killpg(pid, signal.SIGTERM)
    except (ProcessLookupError, PermissionError):
        pass


def start_manager(path: str, cores: int, gpus: int, per_gpu: int, sleep: float) -> int:
    with locked_state(path) as st:
        if pid_alive(st["manager_pid"]):
            return st["manager_pid"]
        cmd = [sys.executable, os.path.abspath(__file__), "--manager", "-f", path, "-c", str(cores),
               "-g", str(gpus), "--per-gpu", str(per_gpu), "-t", str(sleep)]
        p = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                             start_new_session=True)
        st["manager_pid"] = p.pid
        return p.pid


def kill_all(path: str) -> int:
    n = 0
    with locked_state(path) as st:
        st["manager_pid"] = 0
        for j in st["jobs"].values():
            if j["state"] == RUNNING and pid_alive(j["pid"]):
                _kill_group(j["pid"])
                n += 1
            if j["state"] in (RUNNING, QUEUED):
                j["state"] = KILLED
                j["ended"] = time.time()
    return n


def wait_all(path: str, timeout: float = 0, sleep: float = 0.2) -> bool:
    t0 = time.time()
    while True:
        st = read_state(path)
        pending = [j for j in st["jobs"].values() if j["state"] in (QUEUED, RUNNING)]
        if not pending:
            return True
        if pending and not pid_alive(st["manager_pid"]) and all(j["state"] == QUEUED for j in pending):
            return False   # nobody will run them
        if timeout and time.time() - t0 > timeout:
            return False
        time.sleep(sleep)


def job_state(path: str, jid: int) -> Optional[Dict]:
    return read_state(path)["jobs"].get(str(jid))


def print_state(path: str) -> None:
    st = read_state(path)
    print(f"manager pid: {st['manager_pid']} ({'alive' if pid_alive(st['manager_pid']) else 'not running'})")
    print(f"{'id':>6} {'state':<9} {'slot':>4} {'rc':>4} {'runtime':>8}  script")
    for k in sorted(st["jobs"], key=int):
        j = st["jobs"][k]
        rt = ""
        if j["started"]:
            rt = f"{(j['ended'] or time.time()) - j['started']:.1f}s"
        print(f"{k:>6} {j['state']:<9} {str(j['slot'] if j['slot'] is not None else '-'):>4} "
              f"{str(j['rc'] if j['rc'] is not None else '-'):>4} {rt:>8}  {j['script']}")


def self_test() -> int:
    d = tempfile.mkdtemp(prefix="procman_selftest_")
    path = os.path.join(d, "state.json")
    scripts = []
    for i in range(6):
        s = os.path.join(d, f"job{i}.sh")
        with open(s, "w") as f:
            f.write(f"sleep 0.{i}\necho slot=$ASIM_SLOT job=$PROCMAN_JOB_ID > out{i}.txt\n" +
                    ("exit 3\n" if i == 5 else ""))
        scripts.append(s)
    ids = submit(path, scripts)
    start_manager(path, cores=3, gpus=0, per_gpu=1, sleep=0.05)
    ok = wait_all(path, timeout=60)
    st = read_state(path)["jobs"]
    good = ok and all(st[str(i)]["state"] == DONE for i in ids[:5]) and st[str(ids[5])]["state"] == FAILED \
        and st[str(ids[5])]["rc"] == 3 and all(os.path.exists(os.path.join(d, f"out{i}.txt")) for i in range(6)) \
        and len({st[str(i)]["slot"] for i in ids}) <= 3
    print("procman self test", "PASSED" if good else "FAILED")
    if not good:
        print(json.dumps(st, indent=1))
    return 0 if good else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("scripts", nargs="*")
    ap.add_argument("-s", "--selfTest", action="store_true")
    ap.add_argument("-f", "--file", default=default_state_file())
    ap.add_argument("-t", "--sleepTime", type=float, default=0.5)
    ap.add_argument("-c", "--cores", type=int, default=os.cpu_count() or 1)
    ap.add_argument("-g", "--gpus", type=int, default=int(os.environ.get("PROCMAN_GPUS", "0")),
                    help="GPU slots: jobs get HIP_VISIBLE_DEVICES=<gpu> (0 = CPU-only scheduling)")
    ap.add_argument("--per-gpu", type=int, default=int(os.environ.get("PROCMAN_PER_GPU", "2")),
                    help="concurrent jobs per GPU")
    ap.add_argument("-S", "--start", action="store_true")
    ap.add_argument("-p", "--printState", action="store_true")
    ap.add_argument("-k", "--kill", action="store_true")
    ap.add_argument("-j", "--procManForJob", type=int, default=None)
    ap.add_argument("-w", "--wait", action="store_true")
    ap.add_argument("--manager", action="store_true", help=argparse.SUPPRESS)
    o = ap.parse_args(argv)
    if o.selfTest:
        return self_test()
    if o.manager:
        manager_loop(o.file, o.cores, o.gpus, o.per_gpu, o.sleepTime)
        return 0
    if o.scripts:
        for jid in submit(o.file, o.scripts, cwd=os.getcwd()):
            print(jid)
    if o.start:
        start_manager(o.file, o.cores, o.gpus, o.per_gpu, o.sleepTime)
    if o.kill:
        print(f"killed {kill_all(o.file)} running jobs")
    if o.procManForJob is not None:
        j = job_state(o.file, o.procManForJob)
        if j is None:
            print(f"job {o.procManForJob} unknown to {o.file}")
            return 1
        print(f"{o.file} {j['state']}")
    if o.printState:
        print_state(o.file)
    if o.wait:
        return 0 if wait_all(o.file) else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
