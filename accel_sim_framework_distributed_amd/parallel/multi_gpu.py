"""Multi-GPU simulation: one simulated GPU per MI355X rank.

The reference's "distributed" fork only adds a constant latency per
ncclAllReduce to a single simulated GPU (gpu-simulator/main.cc:116-122).
Here every rank simulates its own GPU.  At each collective the ranks either

* ``packet`` (default): run the packet-level link model together, exchanging
  link packets every lookahead epoch with an all-to-all over RCCL/xGMI
  (parallel/collectives.py, csrc/parallel/linksim.h); or
* ``ring``/``tree``/``const``: synchronise their simulated clocks (MAX of the
  arrival cycles over RCCL) and charge the analytic cost after the last rank
  arrives (CollectiveSync).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from .. import _native
from ..sim import build_args
from .collectives import PacketCollective


class CollectiveSync:
    """Collective hook: max-reduce arrival cycles across ranks, then add the
    modelled collective duration."""

    def __init__(self, world: int):
        self.world = world
        self.events: List[Dict] = []

    def __call__(self, sim, desc: Dict, now: int) -> int:
        import torch
        import torch.distributed as dist
        arrive = now
        if self.world > 1 and dist.is_available() and dist.is_initialized():
            on_dev = torch.cuda.is_available() and dist.get_backend() == "nccl"
            dev = torch.device("cuda", torch.cuda.current_device()) if on_dev else torch.device("cpu")
            t = torch.tensor([float(now)], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            arrive = int(t.item())
        line = desc["text"]
        cost = int(sim.collective_cycles(line))
        self.events.append(dict(op=desc["op"], now=now, arrive=arrive, cost=cost))
        return (arrive - now) + cost


class DistributedSuite:
    """Runs a directory of applications (``<root>/<app>/<args>/traces``)."""

    def __init__(self, root: str, config: str = "QV100", engine: str = "gpu", rank: int = 0, world: int = 1,
                 apps: Optional[List[str]] = None, verbose: bool = False, collective_model: str = "packet"):
        self.mod = _native.load(prefer_torch_runtime=True)
        self.root = root
        self.config = config
        self.engine = engine
        self.rank = rank
        self.world = world
        self.verbose = verbose
        self.collective_model = collective_model
        self.apps = []
        for app in sorted(os.listdir(root)):
            if app.startswith("all-reduce") or app.startswith("dp-step") or app.startswith("."):
                continue
            if apps and app not in apps:
                continue
            d = os.path.join(root, app)
            for args in sorted(os.listdir(d)):
                kl = os.path.join(d, args, "traces", "kernelslist.g")
                if os.path.exists(kl):
                    self.apps.append((app, kl))
        self.max_concurrency = None
        self.plan_source = "local"
        self.weights: Dict[str, float] = {}  # last wall time per app (LPT order)
        self.times: Dict = {}                # (app, engine) -> last wall time
        self.assignment: Dict[str, str] = {}
        # the all-reduce example traced for this rank count (all-reduce-<N>),
        # or the single-rank one
        ar = os.path.join(root, f"all-reduce-{world}", "kernelslist.g")
        if not os.path.exists(ar):
            ar = os.path.join(root, "all-reduce", "kernelslist.g")
        self.allreduce = ar if os.path.exists(ar) else None
        # one data-parallel training step per rank (tracegen/training.py):
        # per-layer gradient all-reduces on a communication stream overlapping
        # the backward pass; it replaces the all-reduce example when present
        dp = os.path.join(root, f"dp-step-{world}", f"rank{rank}", "kernelslist.g")
        self.dp_step = dp if os.path.exists(dp) and (not apps or "dp-step" in apps) else None
        self.dp_last: Dict = {}
        self.calibration: Dict = {}
        self.predicted_span = 0.0
        if self.dp_step:
            # scheduled like any application (node placement, LPT order)
            self.apps.append(("dp-step", self.dp_step))
        self._calibrating = False
        # host threads of each application simulated on the CPU engine
        # (-sim_cpu_threads: the engine's persistent thread team); node mode
        # widens the applications on the critical path when cores are spare
        self.threads: Dict[str, int] = {}
        self.sync = PacketCollective() if collective_model == "packet" else CollectiveSync(world)
        # HIP's current device is per host thread: worker threads start on
        # device 0, so every thread this suite creates binds this rank's GPU
        # first (else all ranks of a node would simulate on GPU 0)
        self.device_index = None
        try:
            import torch
            if torch.cuda.is_available():
                self.device_index = torch.cuda.current_device()
        except Exception:  # pragma: no cover - torch is optional for the CPU engine
            pass

    @staticmethod
    def mock_gpu() -> bool:
        """``ASIM_MOCK_GPU=1``: the CPU tier's stand-in for the GPU engine (it
        runs the bit-identical CPU engine under the GPU engine's name, with
        ``ASIM_MOCK_GPU_SLOTS`` concurrent slots), so the node planner and the
        multi-rank plan agreement run in CPU-only tests."""
        return os.environ.get("ASIM_MOCK_GPU", "0") not in ("", "0")

    def _dist(self):
        try:
            import torch.distributed as dist
            if self.world > 1 and dist.is_available() and dist.is_initialized():
                return dist
        except Exception:  # pragma: no cover - torch is optional for the CPU engine
            pass
        return None

    def agree_plan(self) -> bool:
        """Every rank runs rank 0's placement (engine and host threads per
        application, and the timings that order them).  Ranks calibrate under
        their own host load, so independent plans could differ; the step of a
        multi-GPU run must be one plan.  Returns whether this rank's own plan
        already matched rank 0's."""
        dist = self._dist()
        mine = dict(assignment=dict(self.assignment), threads=dict(self.threads))
        if dist is None:
            self.plan_source = "local"
            return True
        obj = [dict(assignment=self.assignment, threads=self.threads, times=self.times,
                    predicted_span=self.predicted_span) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        r0 = obj[0]
        same = r0["assignment"] == mine["assignment"] and r0["threads"] == mine["threads"]
        self.assignment = dict(r0["assignment"])
        self.threads = dict(r0["threads"])
        self.times.update(r0["times"])
        self.predicted_span = r0["predicted_span"]
        self.plan_source = "rank0"
        return same

    def gather(self, info: Dict) -> List[Dict]:
        """`info` of every rank, at every rank (all_gather_object), rank order."""
        dist = self._dist()
        if dist is None:
            return [info]
        out = [None] * self.world
        dist.all_gather_object(out, info)
        return out

    def _bind_device(self):
        if self.device_index is not None:
            import torch
            torch.cuda.set_device(self.device_index)

    def _sim(self, kl: str, engine: Optional[str] = None, threads: int = 1):
        extra = {"-collective_model": self.collective_model}
        eng = engine or ("gpu" if self.engine == "node" else self.engine)
        if eng == "gpu" and self.mock_gpu():
            eng = "cpu"
        if eng == "cpu" and threads > 1:
            extra["-sim_cpu_threads"] = str(threads)
        args = build_args(self.config, kl, eng, extra)
        return self.mod.Simulator(args, self.verbose)

    def concurrency(self) -> int:
        """Simulations that run at once.  GPU engine: as many as fit on this
        GPU (each needs all its unit blocks co-resident).  CPU engine: job
        level parallelism, one single-threaded simulation per host core
        (``ASIM_CPU_JOBS`` overrides the core count)."""
        if self.engine == "cpu":
            n = self.cpu_slots()
            return max(1, min(len(self.apps) or 1, n))
        if self.mock_gpu():
            return max(1, int(os.environ.get("ASIM_MOCK_GPU_SLOTS", "2")))
        cus = int(self.mod.gpu_cu_count())
        cfg = self.mod.parse_config(build_args(self.config, None, "cpu"))
        per = self.mod.gpu_cus_per_sim(cfg["n_sm"], cfg["n_mem"]) if hasattr(self.mod, "gpu_cus_per_sim") \
            else cfg["n_sm"] + cfg["n_mem"]
        # ASIM_GPU_BLOCKS caps a simulation's blocks (units time-slice over them)
        cap = int(os.environ.get("ASIM_GPU_BLOCKS", "0") or 0)
        if cap > 0:
            per = min(per, cap)
        return max(1, cus // per // self.ranks_per_gpu()) if cus else 1

    @staticmethod
    def gpu_reserve(gslots: int) -> int:
        """Host cores kept for the threads driving GPU-engine simulations.
        They sleep while their launches run (a blocking-sync event in
        gpu_engine.hip) and work only between launches (trace ingest, kernel
        setup), so a few cores cover them however many run: half the GPU
        slots, at least one, at most ASIM_GPU_HOST_RESERVE (default 2)."""
        cap = max(1, int(os.environ.get("ASIM_GPU_HOST_RESERVE", "2")))
        return max(1, min(gslots, cap, (gslots + 1) // 2))

    def cpu_slots(self, reserve: int = 0) -> int:
        """Host cores this rank may use for CPU-engine simulations: its share
        of the node's cores (ranks of one node split them), less `reserve`
        (the host threads driving GPU-engine simulations).  ``ASIM_CPU_JOBS``
        overrides."""
        n = int(os.environ.get("ASIM_CPU_JOBS", "0") or 0)
        if n <= 0:
            try:
                n = len(os.sched_getaffinity(0))
            except AttributeError:  # pragma: no cover - non-Linux
                n = os.cpu_count() or 1
            q = self.cgroup_cores()
            if q:
                n = min(n, q)
            # one GPU's share of the node: a rank gets the same cores whether
            # its node runs 1 rank or one per visible GPU (weak scaling keeps
            # the per-GPU resources fixed)
            n //= max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")), self.visible_gpus())
        return max(1, n - reserve)

    @staticmethod
    def visible_gpus() -> int:
        """GPUs this process can see (device count only: no HIP context)."""
        try:
            import torch
            return int(torch.cuda.device_count())
        except Exception:  # pragma: no cover - torch is optional for the CPU engine
            return 0

    @staticmethod
    def cgroup_cores() -> int:
        """Cores the cgroup's CPU quota grants (cgroup v2 cpu.max), 0 when
        unlimited or unknown: the affinity mask can list every core of a
        machine whose quota is a fraction of them."""
        try:
            with open("/sys/fs/cgroup/cpu.max") as f:
                q, per = f.read().split()[:2]
            if q == "max":
                return 0
            return max(1, -(-int(q) // int(per)))
        except (OSError, ValueError):
            return 0

    _rpg_cache: Optional[int] = None

    @classmethod
    def ranks_per_gpu(cls) -> int:
        """Ranks of this node that share one physical GPU (1 in production:
        one rank per MI355X).  Co-resident simulations of ranks sharing a card
        must split its CUs.  Decided from the devices' identities (host name +
        PCI bus id, gathered over the process group), never from how many
        devices a rank can see: with HIP_VISIBLE_DEVICES every rank sees one.
        ``ASIM_RANKS_PER_GPU`` overrides."""
        env = os.environ.get("ASIM_RANKS_PER_GPU")
        if env:
            return max(1, int(env))
        if cls._rpg_cache is not None:
            return cls._rpg_cache
        n = 1
        try:
            import socket
            import torch
            import torch.distributed as dist
            if torch.cuda.is_available() and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                p = torch.cuda.get_device_properties(torch.cuda.current_device())
                ident = getattr(p, "uuid", None) or getattr(p, "pci_bus_id", None)
                me = (socket.gethostname(), str(ident), getattr(p, "pci_bus_id", -1), getattr(p, "pci_domain_id", -1))
                allids = [None] * dist.get_world_size()
                dist.all_gather_object(allids, me)
                n = max(1, sum(1 for x in allids if x == me))
        except Exception:  # pragma: no cover - identity unavailable: assume one rank per GPU
            n = 1
        cls._rpg_cache = n
        return n

    def _run_app(self, app_kl, engine: Optional[str] = None):
        import time
        app, kl = app_kl
        t0 = time.perf_counter()
        if app == "dp-step":
            r = self._run_dp_step(engine, coupled=not self._calibrating)
            dt = time.perf_counter() - t0
            self.weights[app] = dt
            self.times[(app, engine or ("gpu" if self.engine == "node" else self.engine))] = dt
            return r
        eng = engine or ("gpu" if self.engine == "node" else self.engine)
        s = self._sim(kl, engine, self.threads.get(app, 1) if eng == "cpu" else 1)
        rc = s.run()
        if rc != 0:
            raise RuntimeError(f"{app}: simulation failed (deadlock={s.deadlock})\n{s.output[-1500:]}")
        dt = time.perf_counter() - t0
        self.weights[app] = dt
        self.times[(app, engine or ("gpu" if self.engine == "node" else self.engine))] = dt
        return app, s.tot_insn, s.tot_cycle

    # ---- whole-node mode: GPU-engine slots and CPU-engine cores together ----
    # A cycle-level simulation is a long chain of dependent epochs.  The HIP
    # engine wins where an epoch carries much parallel work (many busy SMs:
    # hotspot, heartwall, backprop); a latency-bound application (few warps,
    # many short kernels: bfs, nw, streamcluster) runs about as fast on one
    # host core.  The node schedule gives every application the engine that
    # minimises the step's makespan, like the reference's job-level
    # parallelism (procman over a node's cores) plus the GPU.
    def calibrate(self, rounds: int = 2) -> Dict[str, Dict[str, float]]:
        """Time every application on both engines (GPU slots and CPU cores
        side by side), so plan() can place them.  Each (application, engine)
        keeps its fastest of `rounds` timings: one sample taken under the
        whole node's load is noisy enough to flip a placement."""
        from concurrent.futures import ThreadPoolExecutor
        gslots = max(1, self.concurrency())
        cslots = self.cpu_slots(reserve=self.gpu_reserve(gslots))
        best: Dict = {}
        # the DDP step is timed uncoupled (its collectives emulated locally):
        # two engines running it at once must not both talk to the other ranks
        self._calibrating = True
        try:
            for _ in range(max(1, rounds)):
                with ThreadPoolExecutor(max_workers=gslots, initializer=self._bind_device) as gx, \
                        ThreadPoolExecutor(max_workers=cslots) as cx:
                    fg = [gx.submit(self._run_app, a, "gpu") for a in self.apps]
                    fc = [cx.submit(self._run_app, a, "cpu") for a in self.apps]
                    for f in fg + fc:
                        f.result()
                for a, _ in self.apps:
                    for e in ("gpu", "cpu"):
                        best[(a, e)] = min(best.get((a, e), float("inf")), self.times[(a, e)])
        finally:
            self._calibrating = False
        self.times.update(best)
        self.calibration = {a: {"gpu": round(self.times[(a, "gpu")], 4), "cpu": round(self.times[(a, "cpu")], 4)}
                            for a, _ in self.apps}
        return self.calibration

    @staticmethod
    def _lpt(ts: List[float], slots: int) -> float:
        load = [0.0] * max(1, slots)
        for t in sorted(ts, reverse=True):
            i = min(range(len(load)), key=load.__getitem__)
            load[i] += t
        return max(load) if ts else 0.0

    @staticmethod
    def _cores_span(jobs: List, cores: int) -> float:
        """Makespan of (seconds, threads) jobs list-scheduled longest first on
        `cores` host cores (a job starts when its threads' cores are free)."""
        free = [0.0] * max(1, cores)
        end = 0.0
        for t, k in sorted(jobs, key=lambda x: -x[0]):
            k = max(1, min(k, len(free)))
            free.sort()
            start = free[k - 1]
            for i in range(k):
                free[i] = start + t
            end = max(end, start + t)
        return end

    def plan(self):
        """Engine per application minimising the predicted makespan
        (exhaustive over the subsets sent to the GPU; LPT over the GPU slots,
        list scheduling over the host cores with each CPU application's
        thread count)."""
        gslots = max(1, self.concurrency())
        cslots = self.cpu_slots(reserve=self.gpu_reserve(gslots))
        names = [a for a, _ in self.apps]
        tg = [self.times.get((a, "gpu"), 1.0) for a in names]
        tc = [self.times.get((a, "cpu"), 1.0) for a in names]
        th = [self.threads.get(a, 1) for a in names]
        n = len(names)
        spans = []
        for m in range(1 << n) if n <= 16 else [(1 << n) - 1]:
            g = [tg[i] for i in range(n) if m >> i & 1]
            c = [(tc[i], th[i]) for i in range(n) if not m >> i & 1]
            spans.append((max(self._lpt(g, gslots), self._cores_span(c, cslots)), m))
        lo = min(sp for sp, _ in spans)
        # among the plans within ASIM_NODE_GPU_TOLERANCE of the shortest
        # makespan, the one that runs the most applications on the GPU engine.
        # Default 0 (exact ties only): on MI355X a 2 % tolerance moved 4 more
        # apps onto the GPU engine, whose concurrent runs then slowed each
        # other -- 205.7 ms/step against 183.7 ms for the pure-makespan plan
        # (profiles/r4/bench_node_r4_gpu_tiebreak.json)
        tol = float(os.environ.get("ASIM_NODE_GPU_TOLERANCE", "0"))
        best = min(((sp, m) for sp, m in spans if sp <= lo * (1.0 + tol)),
                   key=lambda x: (-bin(x[1]).count("1"), x[0]))
        self.assignment = {names[i]: ("gpu" if best[1] >> i & 1 else "cpu") for i in range(n)}
        self.predicted_span = best[0]
        return self.assignment

    def widen(self, max_threads: int = 8, reps: int = 2) -> Dict[str, int]:
        """Give host threads to the CPU-engine application on the critical
        path while cores are spare: double its -sim_cpu_threads, re-time it
        (fastest of `reps`), keep the change if it cut the time by >= 15 %,
        re-plan, repeat.  Stops when the critical path is on the GPU, the
        critical application stops scaling, or the cores run out."""
        gslots = max(1, self.concurrency())
        cores = self.cpu_slots(reserve=self.gpu_reserve(gslots))
        kl_of = dict(self.apps)
        tried = set()
        self._calibrating = True
        try:
            for _ in range(16):
                self.plan()
                cpu_apps = [a for a, e in self.assignment.items() if e == "cpu"]
                gpu_apps = [a for a, e in self.assignment.items() if e == "gpu"]
                crit = max(cpu_apps, key=lambda a: self.times[(a, "cpu")]) if cpu_apps else None
                if crit is None or self.times[(crit, "cpu")] < 0.999 * self.predicted_span:
                    # the GPU side sets the span: offer its longest application
                    # a wider host thread team (the plan moves it if that wins)
                    cand = [a for a in gpu_apps if a not in tried]
                    if not cand:
                        break
                    crit = max(cand, key=lambda a: self.times[(a, "gpu")])
                    cpu_apps = cpu_apps + [crit]
                if crit in tried:
                    break  # the critical app does not scale
                k = self.threads.get(crit, 1)
                nk = min(max_threads, 2 * k)
                used = sum(self.threads.get(a, 1) for a in cpu_apps if a != crit)
                if nk <= k or used + nk > cores:
                    break
                old = self.times[(crit, "cpu")]
                # the doubled team, and if that alone does not pay, the team
                # doubled once more: thread teams often pay only past 2 (the
                # dp step on an MI355X node: 158 -> 140 -> 110 ms at 1 / 2 / 4,
                # tools/dp_step_threads.py)
                ok = False
                wider = 2 * nk <= max_threads and os.environ.get("ASIM_NODE_WIDEN_WIDER", "1") != "0"
                for team in [nk] + ([2 * nk] if wider else []):
                    if used + team > cores:
                        break
                    self.threads[crit] = team
                    t = float("inf")
                    for _r in range(max(1, reps)):
                        self._run_app((crit, kl_of[crit]), "cpu")
                        t = min(t, self.times[(crit, "cpu")])
                    if t <= 0.85 * old:
                        self.times[(crit, "cpu")] = t
                        ok = True
                        break
                if not ok:
                    self.threads[crit] = k
                    self.times[(crit, "cpu")] = old
                    tried.add(crit)
        finally:
            self._calibrating = False
        self.plan()
        return {a: k for a, k in self.threads.items() if k > 1}

    def _step_node(self):
        import threading
        from concurrent.futures import ThreadPoolExecutor
        if not getattr(self, "assignment", None):
            if not all((a, e) in self.times for a, _ in self.apps for e in ("gpu", "cpu")):
                self.calibrate()
                self.widen()
            self.plan()
        gslots = max(1, self.concurrency())
        cslots = self.cpu_slots(reserve=self.gpu_reserve(gslots))
        ga = sorted([x for x in self.apps if self.assignment[x[0]] == "gpu"], key=lambda x: -self.times[(x[0], "gpu")])
        ca = sorted([x for x in self.apps if self.assignment[x[0]] == "cpu"], key=lambda x: -self.times[(x[0], "cpu")])
        # host cores as tokens: an application takes its threads' worth before
        # it starts, so thread teams never oversubscribe the cores
        cv = threading.Condition()
        free = [cslots]

        def run_cpu(a):
            k = max(1, min(self.threads.get(a[0], 1), cslots))
            with cv:
                cv.wait_for(lambda: free[0] >= k)
                free[0] -= k
            try:
                return self._run_app(a, "cpu")
            finally:
                with cv:
                    free[0] += k
                    cv.notify_all()

        with ThreadPoolExecutor(max_workers=gslots, initializer=self._bind_device) as gx, \
                ThreadPoolExecutor(max_workers=max(1, min(cslots, len(ca) or 1))) as cx:
            fg = [gx.submit(self._run_app, a, "gpu") for a in ga]
            fc = [cx.submit(run_cpu, a) for a in ca]
            return [f.result() for f in fg + fc]

    def _run_allreduce(self):
        s = self._sim(self.allreduce)
        s.set_collective_hook(lambda d, now, s=s: self.sync(s, d, now))
        if s.run() != 0:
            raise RuntimeError("all-reduce example failed\n" + s.output[-1500:])
        return "all-reduce", s.tot_insn, s.tot_cycle

    def _run_dp_step(self, engine: Optional[str] = None, coupled: bool = True):
        """The rank's DDP step with concurrent kernels: its all-reduces start
        when the layer's gradient is ready and couple this rank's simulated
        clock to the others' mid-step (packet link model over RCCL).
        Uncoupled (calibration), the simulator emulates all ranks locally."""
        self._bind_device()
        # the all-reduces' buffer traffic (RCCL-style copy kernels) runs through
        # the simulated L2 / HBM and contends with the backward kernels
        extra = {"-collective_model": self.collective_model, "-gpgpu_concurrent_kernel_sm": "1",
                 "-collective_mem_traffic": "1"}
        eng = engine or ("gpu" if self.engine == "node" else self.engine)
        if eng == "cpu" and self.threads.get("dp-step", 1) > 1:
            extra["-sim_cpu_threads"] = str(self.threads["dp-step"])
        if eng == "gpu" and self.mock_gpu():
            eng = "cpu"
        s = self.mod.Simulator(build_args(self.config, self.dp_step, eng, extra), self.verbose)
        n0 = len(getattr(self.sync, "events", []))
        if coupled:
            s.set_collective_hook(lambda d, now, s=s: self.sync(s, d, now))
        if s.run() != 0:
            raise RuntimeError("dp step failed\n" + s.output[-1500:])
        ev = getattr(self.sync, "events", [])[n0:] if coupled else []
        if not coupled:
            return "dp-step", s.tot_insn, s.tot_cycle
        ks = s.kernels
        comp = sum(k["cycles"] for k in ks)
        self.dp_last = dict(cycles=int(s.tot_cycle), kernels=len(ks), collectives=len(s.collectives),
                            comm_cycles=int(sum(c["cycles"] for c in s.collectives)), kernel_cycles=int(comp),
                            modes=sorted({e.get("mode", "") for e in ev}))
        return "dp-step", s.tot_insn, s.tot_cycle

    def step(self) -> Dict:
        insn = cycles = 0
        per_app = {}
        conc = self.concurrency() if self.max_concurrency is None else self.max_concurrency
        if self.engine == "node":
            results = self._step_node()
        elif conc <= 1:
            results = [self._run_app(x) for x in self.apps]
        else:
            from concurrent.futures import ThreadPoolExecutor
            # longest (by last measured wall time) first: greedy LPT over the CU groups
            order = sorted(self.apps, key=lambda x: -self.weights.get(x[0], 0.0))
            with ThreadPoolExecutor(max_workers=conc, initializer=self._bind_device) as ex:
                results = list(ex.map(self._run_app, order))
        # The all-reduce example closes the step on the main thread.  (Packing
        # it into the suite's thread pool, or running it beside the pool,
        # measured 3-15 % slower per step on one MI355X: its two kernels then
        # compete with the suite for the CU pool.)
        if self.allreduce and not self.dp_step:
            results.append(self._run_allreduce())
        insn_gpu = 0
        for app, i, c in results:
            insn += i
            cycles += c
            eng = self.engine_of(app)
            if eng == "gpu":
                insn_gpu += i
            per_app[app] = dict(insn=i, cycles=c, wall_s=self.weights.get(app, 0.0), engine=eng)
        return dict(insn=insn, cycles=cycles, insn_gpu=insn_gpu, apps=per_app)

    def engine_of(self, app: str) -> str:
        """The engine that simulated `app` in the last step."""
        if self.engine == "node":
            return self.assignment.get(app, "cpu") if app != "all-reduce" else "gpu"
        return self.engine
