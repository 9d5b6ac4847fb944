"""Loader for the in-tree native module ``_asim`` (built by build_native.py)."""
from __future__ import annotations

import importlib
import os
import sys

_mod = None
_dist = None


def load(prefer_torch_runtime: bool = False):
    """Import the native module.

    ``prefer_torch_runtime``: import torch first so the process binds the HIP
    runtime bundled with PyTorch (same SONAME as /opt/rocm's); required when
    the simulator shares a process with torch.distributed / RCCL.
    """
    global _mod
    if _mod is not None:
        return _mod
    if prefer_torch_runtime:
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is optional here
            pass
    alt = os.environ.get("ASIM_NATIVE_SO")
    if alt:
        # A/B runs inside one GPU call: another build of the same module
        # (e.g. the previous commit's) loaded from its own file
        from importlib import util as ilu
        spec = ilu.spec_from_file_location("accel_sim_framework_distributed_amd._asim", alt)
        m = ilu.module_from_spec(spec)
        spec.loader.exec_module(m)
        sys.modules["accel_sim_framework_distributed_amd._asim"] = m
        _mod = m
        return _mod
    try:
        _mod = importlib.import_module("accel_sim_framework_distributed_amd._asim")
    except ImportError as e:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        raise ImportError(
            "native module _asim is not built; run `python build_native.py` in " + root + f" ({e})") from e
    return _mod


def gpu_available() -> bool:
    return bool(load().gpu_available())


def load_dist():
    """The native epoch loop of the packet collective (``_asim_dist``, a torch
    C++ extension built in-tree by build_native.py), or None if it is not
    built (the Python loop of parallel/collectives.py is used then)."""
    global _dist
    if _dist is not None:
        return _dist or None
    import importlib.util
    import torch  # noqa: F401  (the extension links libtorch)
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_asim_dist.so")
    if not os.path.exists(p):
        _dist = False
        return None
    spec = importlib.util.spec_from_file_location("_asim_dist", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    _dist = m
    return m
