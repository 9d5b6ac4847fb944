"""Front-end of the MI355X cycle engine (csrc/engine/gpu_engine.hip).

The framework's device "ops" are the persistent HIP kernel that advances a
simulated GPU epoch by epoch (one 64-lane wavefront per simulated SM or memory
channel, csrc/engine) and the CDNA4 micro-benchmarks (csrc/ubench).  This
module reports how the engine kernel was compiled and how it occupies the
chip; `ubench.py` runs the micro-benchmarks.
"""
from __future__ import annotations

from typing import Dict

from .. import _native


def kernel_info() -> Dict[str, int]:
    """Compiled resources of the engine kernel (VGPRs, scratch, LDS) and the
    per-block state sizes; empty without a usable HIP device."""
    mod = _native.load(prefer_torch_runtime=True)
    if not mod.gpu_available():
        return {}
    return dict(mod.gpu_engine_kernel_info())


def footprint(config: str = "QV100") -> Dict[str, int]:
    """How one simulation of `config` occupies an MI355X: units (simulated
    SMs + memory channels), blocks (one wavefront each; the LDS-state build
    fits one per CU, the default split-state build several: the CUs a
    simulation reserves come from the native engine, gpu_cus_per_sim), and
    how many such simulations fit side by side on the device."""
    from ..sim import build_args
    mod = _native.load(prefer_torch_runtime=True)
    cfg = mod.parse_config(build_args(config, None, "cpu"))
    units = int(cfg["n_sm"]) + int(cfg["n_mem"])
    cus = int(mod.gpu_cu_count()) if mod.gpu_available() else 0
    blocks = min(units, cus) if cus else units
    per = int(mod.gpu_cus_per_sim(int(cfg["n_sm"]), int(cfg["n_mem"]))) if cus else 0
    return dict(sm_blocks=int(cfg["n_sm"]), channel_blocks=int(cfg["n_mem"]), units=units, blocks=blocks,
                units_per_block=-(-units // blocks), device_cus=cus, cus_per_simulation=per,
                concurrent_simulations=(cus // per) if per else 0, epoch_cycles=int(cfg["icnt_latency"]))
