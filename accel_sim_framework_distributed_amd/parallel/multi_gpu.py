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
            if app.startswith("all-reduce") or app.startswith("."):
                continue
            if apps and app not in apps:
                continue
            d = os.path.join(root, app)
            for args in sorted(os.listdir(d)):
                kl = os.path.join(d, args, "traces", "kernelslist.g")
                if os.path.exists(kl):
                    self.apps.append((app, kl))
        self.max_concurrency = None
        self.weights: Dict[str, float] = {}  # last wall time per app (LPT order)
        # the all-reduce example traced for this rank count (all-reduce-<N>),
        # or the single-rank one
        ar = os.path.join(root, f"all-reduce-{world}", "kernelslist.g")
        if not os.path.exists(ar):
            ar = os.path.join(root, "all-reduce", "kernelslist.g")
        self.allreduce = ar if os.path.exists(ar) else None
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

    def _bind_device(self):
        if self.device_index is not None:
            import torch
            torch.cuda.set_device(self.device_index)

    def _sim(self, kl: str):
        extra = {"-collective_model": self.collective_model}
        args = build_args(self.config, kl, self.engine, extra)
        return self.mod.Simulator(args, self.verbose)

    def concurrency(self) -> int:
        """Simulations that run at once.  GPU engine: as many as fit on this
        GPU (each needs all its unit blocks co-resident).  CPU engine: job
        level parallelism, one single-threaded simulation per host core
        (``ASIM_CPU_JOBS`` overrides the core count)."""
        if self.engine != "gpu":
            n = int(os.environ.get("ASIM_CPU_JOBS", "0") or 0)
            if n <= 0:
                try:
                    n = len(os.sched_getaffinity(0))
                except AttributeError:  # pragma: no cover - non-Linux
                    n = os.cpu_count() or 1
            return max(1, min(len(self.apps) or 1, n))
        cus = int(self.mod.gpu_cu_count())
        cfg = self.mod.parse_config(build_args(self.config, None, "cpu"))
        per = self.mod.gpu_cus_per_sim(cfg["n_sm"], cfg["n_mem"]) if hasattr(self.mod, "gpu_cus_per_sim") \
            else cfg["n_sm"] + cfg["n_mem"]
        return max(1, cus // per // self.ranks_per_gpu()) if cus else 1

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

    def _run_app(self, app_kl):
        import time
        app, kl = app_kl
        t0 = time.perf_counter()
        s = self._sim(kl)
        rc = s.run()
        if rc != 0:
            raise RuntimeError(f"{app}: simulation failed (deadlock={s.deadlock})\n{s.output[-1500:]}")
        self.weights[app] = time.perf_counter() - t0
        return app, s.tot_insn, s.tot_cycle

    def _run_allreduce(self):
        s = self._sim(self.allreduce)
        s.set_collective_hook(lambda d, now, s=s: self.sync(s, d, now))
        if s.run() != 0:
            raise RuntimeError("all-reduce example failed\n" + s.output[-1500:])
        return "all-reduce", s.tot_insn, s.tot_cycle

    def step(self) -> Dict:
        insn = cycles = 0
        per_app = {}
        conc = self.concurrency() if self.max_concurrency is None else self.max_concurrency
        if conc <= 1:
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
        if self.allreduce:
            results.append(self._run_allreduce())
        for app, i, c in results:
            insn += i
            cycles += c
            per_app[app] = dict(insn=i, cycles=c, wall_s=self.weights.get(app, 0.0))
        return dict(insn=insn, cycles=cycles, apps=per_app)
