"""Configuration sweep: every application of the suite under every one of the
tuner's 16 search configurations (BASELINE.json config #5).

The reference's tuner launches the 16 combinations of the four parameters
its micro-benchmarks cannot demystify -- warp scheduler (LRR / GTO), L2
interleaving granularity (32 B / 256 B), partition hashing (linear / IPOLY)
and DRAM scheduler (FR-FCFS / FCFS) -- through run_simulations.py over a
suite (util/tuner/README.md:60-97, util/tuner/tuner.py:15-68,
util/job_launching/run_simulations.py:375-397: one simulator process per
job, queued on the cluster's cores).  Here the same grid is one batch of
independent simulations on one node: the MI355X runs GPU-engine simulations
in its CU groups while the host cores run CPU-engine ones.

Placement (``engine="node"``): both pools pull from one queue ordered by the
applications' measured GPU / CPU time ratio -- GPU slots take jobs from the
GPU-friendly end (many busy SMs per epoch), host cores from the other end --
so the batch ends when both pools run dry.  ``gpu`` / ``cpu`` use one pool.
"""
from __future__ import annotations

import itertools
import threading
import time
from typing import Dict, List, Optional, Tuple

from ..sim import build_args
from ..tuner.tuner import SEARCH_SPACE

# composable extras of job_launching/configs/define-standard-cfgs.yml as flags
EXTRA_FLAGS: Dict[str, Dict[str, str]] = {
    "LINEAR": {"-gpgpu_memory_partition_indexing": "0"},
    "IPOLY": {"-gpgpu_memory_partition_indexing": "2"},
    "RR": {"-gpgpu_scheduler": "lrr"},
    "GTO": {"-gpgpu_scheduler": "gto"},
    # the reference's strings verbatim (define-standard-cfgs.yml:147-151)
    "32B": {"-gpgpu_mem_addr_mapping":
            "dramid@5;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCC.BCCSSSSS"},
    "256B": {"-gpgpu_mem_addr_mapping":
             "dramid@8;00000000.00000000.00000000.00000000.0000RRRR.RRRRRRRR.RBBBCCCB.CCCSSSSS"},
    "FRFCFS": {"-gpgpu_dram_scheduler": "1"},
    "FCFS": {"-gpgpu_dram_scheduler": "0"},
}


def sweep_configs(n: int = 16) -> List[Tuple[str, Dict[str, str]]]:
    """The first `n` of the 16 search combinations: (name, flags)."""
    out = []
    for combo in itertools.product(*SEARCH_SPACE):
        flags: Dict[str, str] = {}
        for t in combo:
            flags.update(EXTRA_FLAGS[t])
        out.append(("-".join(combo), flags))
    return out[:max(1, n)]


class SweepRunner:
    """One batch of (application x configuration) simulations.  `suite` is a
    DistributedSuite (applications, engine pools, calibration)."""

    def __init__(self, suite, n_configs: int = 16):
        self.suite = suite
        self.configs = sweep_configs(n_configs)
        self.jobs = [(a, kl, cname, flags) for (a, kl) in suite.apps if a != "dp-step"
                     for cname, flags in self.configs]
        self.ratio: Dict[str, float] = {}
        self.cpu_s: Dict[str, float] = {}  # calibration: one host core's time per application
        self.last: Dict = {}

    def calibrate(self) -> Dict[str, float]:
        """GPU / CPU wall-time ratio of every application (its base config,
        one untimed run per engine): the queue order."""
        s = self.suite
        if s.engine == "node":
            for (a, kl) in s.apps:
                if a == "dp-step":
                    continue
                t = {}
                for eng in ("gpu", "cpu"):
                    t0 = time.perf_counter()
                    self._run(a, kl, {}, eng)
                    t[eng] = time.perf_counter() - t0
                self.ratio[a] = t["gpu"] / max(t["cpu"], 1e-9)
                self.cpu_s[a] = t["cpu"]
        return dict(self.ratio)

    def gpu_takes(self, job, rest, cslots: int) -> bool:
        """Node placement at the queue's GPU end: a GPU slot takes `job` while
        the GPU would finish it no later than the host cores would get to it
        and finish it themselves (one core's time, or the time the cores need
        for everything still queued, whichever is longer).  Near the end of a
        sweep the host cores run out of work first; a slow GPU job taken then
        would be the step's tail."""
        if cslots <= 0 or job[0] not in self.cpu_s:
            return True
        cpu = self.cpu_s[job[0]]
        drain = sum(self.cpu_s.get(j[0], cpu) for j in rest) / cslots
        return self.ratio.get(job[0], 1.0) * cpu <= max(cpu, drain)

    def _run(self, app: str, kl: str, flags: Dict[str, str], eng: str):
        s = self.suite
        extra = {"-collective_model": s.collective_model, **flags}
        e = "cpu" if (eng == "gpu" and s.mock_gpu()) else eng
        sim = s.mod.Simulator(build_args(s.config, kl, e, extra), False)
        if sim.run() != 0:
            raise RuntimeError(f"sweep {app} {flags}: simulation failed (deadlock={sim.deadlock})")
        return int(sim.tot_insn), int(sim.tot_cycle)

    def step(self) -> Dict:
        """Run every job once; returns instruction totals per engine."""
        s = self.suite
        mode = s.engine
        gslots = max(1, s.concurrency()) if mode in ("gpu", "node") else 0
        cslots = s.cpu_slots(reserve=s.gpu_reserve(gslots) if mode == "node" else 0) if mode in ("cpu", "node") else 0
        # GPU-friendly first (low gpu/cpu ratio), longest first among equals
        order = sorted(self.jobs, key=lambda j: (self.ratio.get(j[0], 1.0), j[0], j[2]))
        lock = threading.Lock()
        q = list(order)
        tot = {"gpu": [0, 0, 0], "cpu": [0, 0, 0]}  # insn, cycles, jobs
        err: List[BaseException] = []

        def worker(eng: str):
            if eng == "gpu":
                s._bind_device()
            while not err:
                with lock:
                    if not q:
                        return
                    if eng == "gpu" and mode == "node" and not self.gpu_takes(q[0], q, cslots):
                        return  # the rest goes to the host cores
                    job = q.pop(0) if eng == "gpu" else q.pop()
                try:
                    i, c = self._run(job[0], job[1], job[3], eng)
                except BaseException as e:  # noqa: BLE001 - re-raised on the caller's thread
                    err.append(e)
                    return
                with lock:
                    tot[eng][0] += i
                    tot[eng][1] += c
                    tot[eng][2] += 1

        th = [threading.Thread(target=worker, args=("gpu",)) for _ in range(gslots)] + \
             [threading.Thread(target=worker, args=("cpu",)) for _ in range(cslots)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        if err:
            raise err[0]
        self.last = dict(wall_s=dt, gpu_slots=gslots, cpu_slots=cslots,
                         jobs={"gpu": tot["gpu"][2], "cpu": tot["cpu"][2]})
        return dict(insn=tot["gpu"][0] + tot["cpu"][0], insn_gpu=tot["gpu"][0],
                    cycles=tot["gpu"][1] + tot["cpu"][1], jobs=len(self.jobs), wall_s=dt,
                    jobs_gpu=tot["gpu"][2], jobs_cpu=tot["cpu"][2])


__all__ = ["SweepRunner", "sweep_configs", "EXTRA_FLAGS"]
