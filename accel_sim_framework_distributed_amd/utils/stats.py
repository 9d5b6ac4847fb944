"""Parsing of simulator stdout (``key = value`` lines).

The keys are the reference's (gpu-sim.cc:1355-1541 gpu_print_stat,
gpgpusim_entrypoint.cc:248-270 print_simulation_time), so the same regexes
drive get_stats.py, job_status.py and the correlator.
"""
from __future__ import annotations

import re
from typing import Dict, List

_KV = re.compile(r"^\s*([A-Za-z_][\w\[\]\. ]*?)\s*=\s*([-+0-9.eE]+)\s*(%|\(inst/sec\)|\(cycle/sec\)|x|GB/Sec)?\s*$")


def parse_kernels(text: str) -> List[Dict[str, float]]:
    """Split simulator output into per-kernel stat dicts."""
    kernels: List[Dict[str, float]] = []
    cur: Dict[str, float] = {}
    name = None
    for line in text.splitlines():
        if line.startswith("kernel_name"):
            if cur:
                kernels.append(cur)
            cur = {}
            name = line.split("=", 1)[1].strip()
            cur["kernel_name"] = name  # type: ignore[assignment]
            continue
        m = _KV.match(line)
        if not m:
            continue
        key, val, unit = m.group(1).strip(), m.group(2), m.group(3)
        if unit == "(inst/sec)":
            key = "gpgpu_simulation_rate_inst"
        elif unit == "(cycle/sec)":
            key = "gpgpu_simulation_rate_cycle"
        try:
            cur[key] = float(val)
        except ValueError:
            pass
    if cur:
        kernels.append(cur)
    return kernels


def final_stats(text: str) -> Dict[str, float]:
    ks = parse_kernels(text)
    return ks[-1] if ks else {}


def exit_status(text: str) -> str:
    """Classify a run like the reference's job_status.py (status_strings)."""
    if "deadlock detected" in text:
        return "DEADLOCK"
    if "Segmentation fault" in text:
        return "SEGFAULT"
    if "Assertion" in text or "ERROR" in text:
        return "FUNC_TEST_FAILED" if "*** exit detected ***" in text else "ERROR"
    if "*** exit detected ***" in text:
        return "COMPLETE_NO_OTHER_INFO"
    return "RUNNING"
