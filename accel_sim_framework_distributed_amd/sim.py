"""High-level simulator API.

>>> from accel_sim_framework_distributed_amd import sim
>>> r = sim.simulate("traces/kernelslist.g", config="QV100", engine="gpu")
>>> r.tot_insn, r.tot_cycle, r.kips

``config`` is a preset name (models/presets.py), a list of config files
(``-config`` semantics of the reference), or a dict of options.
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, List, Optional, Sequence, Union

from . import _native
from .models import presets
from .utils import stats as _stats

ConfigLike = Union[str, Sequence[str], Dict[str, str]]


def build_args(config: ConfigLike, trace: Optional[str] = None, engine: str = "cpu",
               extra: Optional[Dict[str, str]] = None) -> List[str]:
    args: List[str] = []
    if isinstance(config, str):
        args += presets.args_for(config)
    elif isinstance(config, dict):
        args += presets.args_for(dict(config))
    else:
        for f in config:
            args += ["-config", f]
    if extra:
        for k, v in extra.items():
            args += [k, str(v)]
    if trace:
        args += ["-trace", trace]
    args += ["-sim_engine", engine]
    return args


@dataclasses.dataclass
class SimResult:
    tot_insn: int
    tot_cycle: int
    wall_s: float
    sim_s: float
    kernels: List[Dict]
    collectives: List[Dict]
    output: str
    engine: str
    deadlock: bool

    @property
    def kips(self) -> float:
        """Thousands of simulated (thread) instructions per wall second."""
        return self.tot_insn / max(self.wall_s, 1e-9) / 1e3

    @property
    def stats(self) -> Dict[str, float]:
        return _stats.final_stats(self.output)


class Simulator:
    def __init__(self, config: ConfigLike = "QV100", trace: Optional[str] = None, engine: str = "cpu",
                 extra: Optional[Dict[str, str]] = None, echo: bool = False, torch_runtime: bool = False):
        self.mod = _native.load(prefer_torch_runtime=torch_runtime)
        self.args = build_args(config, trace, engine, extra)
        self.native = self.mod.Simulator(self.args, echo)

    def run(self) -> SimResult:
        t0 = time.perf_counter()
        rc = self.native.run()
        wall = time.perf_counter() - t0
        n = self.native
        if rc != 0 and not n.deadlock:
            raise RuntimeError("simulation failed:\n" + n.output[-2000:])
        return SimResult(n.tot_insn, n.tot_cycle, wall, n.sim_seconds, n.kernels, n.collectives, n.output,
                         n.engine, n.deadlock)


def simulate(trace: str, config: ConfigLike = "QV100", engine: str = "cpu",
             extra: Optional[Dict[str, str]] = None, echo: bool = False) -> SimResult:
    return Simulator(config, trace, engine, extra, echo).run()
