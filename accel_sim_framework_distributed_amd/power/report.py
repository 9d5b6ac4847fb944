"""Parse ``accelwattch_power_report.log`` (one block per kernel)."""
from __future__ import annotations

import re
from typing import Dict, List

COMPONENTS = ["IBP", "ICP", "DCP", "TCP", "CCP", "SHRDP", "RFP", "INTP", "FPUP", "DPUP", "INT_MUL24P", "INT_MUL32P",
              "INT_MULP", "INT_DIVP", "FP_MULP", "FP_DIVP", "FP_SQRTP", "FP_LGP", "FP_SINP", "FP_EXP", "DP_MULP",
              "DP_DIVP", "TENSORP", "TEXP", "SCHEDP", "L2CP", "MCP", "NOCP", "DRAMP", "PIPEP", "IDLE_COREP", "CONSTP",
              "STATICP"]

_KV = re.compile(r"^\s*([A-Za-z0-9_]+)\s*=\s*(\S+)\s*$")


def parse_power_report(path_or_text: str) -> List[Dict[str, float]]:
    """List of kernels: {'kernel_name', 'kernel_launch_uid', 'kernel_avg_power',
    'avg': {component: W}, 'max': {...}, 'min': {...}, 'act': {activity: avg}}."""
    text = path_or_text
    if "\n" not in path_or_text and len(path_or_text) < 4096:
        text = open(path_or_text).read()
    kernels: List[Dict] = []
    cur = None
    for line in text.splitlines():
        m = _KV.match(line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "kernel_name":
            cur = dict(kernel_name=v, avg={}, max={}, min={}, act={}, tot={})
            kernels.append(cur)
            continue
        if cur is None:
            continue
        try:
            x = float(v)
        except ValueError:
            continue
        if k in ("kernel_launch_uid", "gpu_sim_cycle", "kernel_avg_power", "kernel_max_power", "kernel_min_power",
                 "gpu_tot_avg_power", "gpu_tot_max_power", "gpu_tot_min_power", "gpu_avg_threads_per_warp",
                 "kernel_avg_clock_ratio"):
            cur[k] = x
        elif k.startswith("gpu_avg_"):
            n = k[8:]
            (cur["avg"] if n in COMPONENTS else cur["act"])[n] = x
        elif k.startswith("gpu_max_"):
            n = k[8:]
            if n in COMPONENTS:
                cur["max"][n] = x
        elif k.startswith("gpu_min_"):
            n = k[8:]
            if n in COMPONENTS:
                cur["min"][n] = x
        elif k.startswith("gpu_tot_"):
            cur["tot"][k[8:]] = x
    return kernels
