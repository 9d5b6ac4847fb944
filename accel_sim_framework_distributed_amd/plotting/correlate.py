#!/usr/bin/env python3
"""Correlate simulated per-kernel stats with hardware measurements.

Reference: util/plotting/plot-correlation.py (getAppData :32-103 -- error %,
MAE :77-90, Pearson correlation :95, NRMSE :99; options :657-710) and
correl_mappings.py (CorrelStat table).  Inputs here:

* simulation: a ``get_stats.py -k -K`` CSV (rows ``app/args--kernel--N``,
  one column per config);
* hardware: ``hw_stats`` output -- ``<hw_dir>/<app>/<args>/run_<i>/`` with
  rocprofv3 ``*kernel_trace.csv`` files (MI355X) -- or a flat CSV
  ``app,args,kernel,instance,<stat>...`` for data measured elsewhere.

Kernels are matched by launch order within an application; per-app values
are the sum over kernels (the reference's per-app aggregation), and the
headline **cycle MAE** is the mean over apps of |sim - hw| / hw x 100.
Stats are described by Python callables (``CorrelStat``) instead of the
reference's eval'd strings; ``-d`` loads extra mappings from a Python file
defining ``CORREL_STATS``.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import math
import os
import re
import sys
from collections import OrderedDict, defaultdict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.job_launching import get_stats  # noqa: E402
    from accel_sim_framework_distributed_amd.plotting import svg  # noqa: E402
else:
    from ..job_launching import get_stats
    from . import svg


@dataclass
class CorrelStat:
    chart_name: str
    sim_stat: str                                  # get_stats stat regex (block name)
    hw_eval: Callable[[Dict[str, List[float]], float], float]   # (hw columns over runs, clock MHz) -> value
    plotfile: str
    hw_names: Sequence[str] = ()                   # device names this mapping applies to ('' = any)
    drop_hw_below: float = 0.0
    log: bool = True
    sim_scale: float = 1.0
    # derived simulator value: sim_eval({stat regex: per-kernel value}) over
    # sim_stats (sim_stat is then only the chart's key)
    sim_stats: Sequence[str] = ()
    sim_eval: Optional[Callable[[Dict[str, float]], float]] = None
    ratio: bool = False                            # a rate: per-app value is the mean over kernels, not the sum


def _mean(v):
    return float(np.mean(v)) if len(v) else float("nan")


def _median(v):
    return float(np.median(v)) if len(v) else float("nan")


def _hw(*cols: str) -> Callable[[Dict[str, List[float]], float], float]:
    """Sum of the run-mean of rocprofv3 counter columns (NaN if one is absent)."""
    def f(hw, mhz):
        if any(c not in hw for c in cols):
            return float("nan")
        return float(sum(_mean(hw[c]) for c in cols))
    return f


def _hw_ratio(num: Sequence[str], den: Sequence[str], one_minus: bool = False):
    def f(hw, mhz):
        n, d = _hw(*num)(hw, mhz), _hw(*den)(hw, mhz)
        if not (d > 0) or not math.isfinite(n):
            return float("nan")
        r = n / d
        return 1.0 - r if one_minus else r
    return f


def _cycles(hw, mhz):
    return _median(hw["duration_ns"]) * mhz / 1000.0 if "duration_ns" in hw else float("nan")


# simulator stat regexes (they must be listed in job_launching/stats/example_stats.yml)
S_CYC = r"gpu_sim_cycle\s*=\s*(.*)"
S_WINSN = r"gpgpu_n_tot_w_icount\s*=\s*(.*)"
S_LOAD = r"gpgpu_n_load_insn\s*=\s*(.*)"
S_STORE = r"gpgpu_n_store_insn\s*=\s*(.*)"
S_L1 = r"\s+Total_core_cache_stats_breakdown\[%s\]\[%s\]\s*=\s*(.*)"
S_L2 = r"\s+L2_cache_stats_breakdown\[%s\]\[%s\]\s*=\s*(.*)"
S_VALU = r"gpgpu_n_valu_insn\s*=\s*(.*)"
S_SALU = r"gpgpu_n_salu_insn\s*=\s*(.*)"
S_SMEM = r"gpgpu_n_smem_insn\s*=\s*(.*)"
S_VMRD = r"gpgpu_n_vmem_rd_insn\s*=\s*(.*)"
S_VMWR = r"gpgpu_n_vmem_wr_insn\s*=\s*(.*)"
S_LDSI = r"gpgpu_n_lds_insn\s*=\s*(.*)"
S_SQBR = r"gpgpu_n_sq_branch_insn\s*=\s*(.*)"


def _ea_rd_sectors(hw, mhz):
    """TCC->EA read requests in 32 B sectors (requests are 32, 64 or 128 B)."""
    return (_hw("TCC_EA0_RDREQ_32B_sum")(hw, mhz) + 2 * _hw("TCC_EA0_RDREQ_64B_sum")(hw, mhz) +
            4 * _hw("TCC_EA0_RDREQ_128B_sum")(hw, mhz))
_VMEM = ("SQ_INSTS_VMEM_RD_sum", "SQ_INSTS_VMEM_WR_sum")
_WAVE_INSTS = ("SQ_INSTS_VALU_sum", "SQ_INSTS_SALU_sum", "SQ_INSTS_SMEM_sum", "SQ_INSTS_LDS_sum",
               "SQ_INSTS_BRANCH_sum") + _VMEM


_SQ_STATS = (S_VALU, S_SALU, S_SMEM, S_VMRD, S_VMWR, S_LDSI, S_SQBR)


def _ipc(d):
    return d[S_WINSN] / d[S_CYC] if d.get(S_CYC) else float("nan")


S_L1_LK64 = r"\s+L1D_total_64B_tag_lookups\s*=\s*(.*)"


def _l1_hit_rate(d):
    # as the hardware ratio 1 - TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES:
    # read requests the L1 sends over its 64 B tag lookups
    tot = d.get(S_L1_LK64) or 0.0
    return 1.0 - d[S_L1 % ("GLOBAL_ACC_R", "MISS")] / tot if tot else float("nan")


def _l2_hit_rate(d):
    h = _l2_hits(d)
    m = _l2_misses(d)
    return h / (h + m) if h + m else float("nan")


# gfx950's TCC counts every write as a hit: a write allocates its bytes in the
# write-back L2 without fetching the line (byte-masked dirty data), so only
# reads and atomics miss (per app, TCC_HIT + TCC_MISS == TCC_READ + TCC_WRITE
# + TCC_ATOMIC, and TCC_MISS matches the read misses).  The simulator's
# lazy-fetch write allocation ('L' policy) is the same operation, which the
# GPGPU-Sim breakdown files as a write miss; the correlator therefore puts the
# simulator's writes on the hit side and its read / atomic misses on the miss
# side, with the reads merged into a pending miss.
_L2_R_HIT = S_L2 % ("GLOBAL_ACC_R", "HIT")
_L2_W_ALL = S_L2 % ("GLOBAL_ACC_W", "TOTAL_ACCESS")
_L2_R_MISS = S_L2 % ("GLOBAL_ACC_R", "MISS")
_L2_A_MISS = S_L2 % ("GLOBAL_ATOMIC", "MISS")
_L2_R_MSHR = S_L2 % ("GLOBAL_ACC_R", "MSHR_HIT")


def _l2_hits(d):
    return d[_L2_R_HIT] + d[_L2_W_ALL]


def _l2_misses(d):
    # a read merged into a pending miss (the simulator's MSHR hit) waits for
    # the same fill: TCC counts it as a miss
    return d[_L2_R_MISS] + d[_L2_R_MSHR] + d.get(_L2_A_MISS, 0.0)


# Sim statistic <-> MI355X rocprofv3 counter mappings (the reference's
# correl_mappings.py:5-23 maps GPGPU-Sim stats to nvprof/nsight metrics; these
# map the same simulator stats to gfx950 SQ / TCP (L1) / TCC (L2) / EA (HBM)
# counters collected by hw_stats/run_hw.py --counter_groups).
CORREL_STATS: List[CorrelStat] = [
    # median over runs: short kernels on a shared node have a heavy right tail
    CorrelStat("Cycles", S_CYC, _cycles, "cycles"),
    CorrelStat("Instructions (thread)", r"gpu_sim_insn\s*=\s*(.*)",
               lambda hw, mhz: _mean(hw["thread_insts"]) if "thread_insts" in hw else float("nan"), "insn"),
    # the SQ_INSTS_* classes exclude s_waitcnt / s_nop / s_barrier / s_endpgm:
    # the simulator side sums its instructions of the same classes
    CorrelStat("Warp instructions", "warp_insn", _hw(*_WAVE_INSTS), "warp-insn",
               sim_stats=_SQ_STATS, sim_eval=lambda d: sum(d.values())),
    CorrelStat("Warp IPC", "warp_ipc", lambda hw, mhz: _hw(*_WAVE_INSTS)(hw, mhz) / _cycles(hw, mhz),
               "warp-ipc", sim_stats=_SQ_STATS + (S_CYC,),
               sim_eval=lambda d: sum(v for k, v in d.items() if k != S_CYC) / d[S_CYC] if d.get(S_CYC) else float("nan"),
               ratio=True, log=False),
    CorrelStat("Memory instructions (VMEM + LDS)", "mem_insn", _hw(*(_VMEM + ("SQ_INSTS_LDS_sum",))), "mem-insn",
               sim_stats=(S_VMRD, S_VMWR, S_LDSI), sim_eval=lambda d: sum(d.values())),
    CorrelStat("Waves launched", r"gpgpu_n_completed_warps\s*=\s*(.*)", _hw("SQ_WAVES_sum"), "waves"),
    CorrelStat("Branch instructions", r"gpgpu_n_branch_insn\s*=\s*(.*)", _hw("SQ_INSTS_BRANCH_sum"), "branch"),
    CorrelStat("MFMA instructions", r"gpgpu_n_tensor_insn\s*=\s*(.*)", _hw("SQ_INSTS_MFMA_sum"), "mfma"),
    CorrelStat("LDS bank conflict cycles", r"gpgpu_n_shmem_bkconflict\s*=\s*(.*)", _hw("SQ_LDS_BANK_CONFLICT_sum"),
               "lds-conflict"),
    # TCP tag lookups are 64 B: a wave64 dword access (256 B) is 4 of them
    # (per-kernel TCP_TOTAL_CACHE_ACCESSES / VMEM instructions: 4.00 on
    # lud_internal, 1.00 on the 16-lane lud_diagonal)
    CorrelStat("L1 accesses", S_L1_LK64, _hw("TCP_TOTAL_CACHE_ACCESSES_sum"), "l1-acc"),
    CorrelStat("L1 read misses (L1->L2 reads)", S_L1 % ("GLOBAL_ACC_R", "MISS"), _hw("TCP_TCC_READ_REQ_sum"),
               "l1-read-miss"),
    # the write requests the L1 sends (a store may be split into 64 B
    # requests, -sim_l1_write_request_bytes): what arrives at the L2
    CorrelStat("L1->L2 write requests", S_L2 % ("GLOBAL_ACC_W", "TOTAL_ACCESS"), _hw("TCP_TCC_WRITE_REQ_sum"),
               "l1-writes"),
    CorrelStat("L1 read hit rate", "l1_hit_rate",
               _hw_ratio(("TCP_TCC_READ_REQ_sum",), ("TCP_TOTAL_CACHE_ACCESSES_sum",), one_minus=True),
               "l1-hit-rate", sim_stats=(S_L1 % ("GLOBAL_ACC_R", "MISS"), S_L1_LK64),
               sim_eval=_l1_hit_rate, ratio=True, log=False),
    CorrelStat("L2 read accesses", S_L2 % ("GLOBAL_ACC_R", "TOTAL_ACCESS"), _hw("TCC_READ_sum"), "l2-reads"),
    CorrelStat("L2 write accesses", S_L2 % ("GLOBAL_ACC_W", "TOTAL_ACCESS"), _hw("TCC_WRITE_sum"), "l2-writes"),
    CorrelStat("L2 atomic accesses", S_L2 % ("GLOBAL_ATOMIC", "TOTAL_ACCESS"), _hw("TCC_ATOMIC_sum"), "l2-atomics"),
    CorrelStat("L2 hits", "l2_hits", _hw("TCC_HIT_sum"), "l2-hits",
               sim_stats=(_L2_R_HIT, _L2_W_ALL), sim_eval=_l2_hits),
    CorrelStat("L2 misses", "l2_misses", _hw("TCC_MISS_sum"), "l2-misses",
               sim_stats=(_L2_R_MISS, _L2_R_MSHR), sim_eval=_l2_misses),
    CorrelStat("L2 hit rate", "l2_hit_rate", _hw_ratio(("TCC_HIT_sum",), ("TCC_HIT_sum", "TCC_MISS_sum")),
               "l2-hit-rate", sim_stats=(_L2_R_HIT, _L2_R_MSHR, _L2_W_ALL, _L2_R_MISS),
               sim_eval=_l2_hit_rate, ratio=True, log=False),
    # requests leaving the L2 for the Infinity Fabric (MALL, then HBM): the
    # deepest level rocprofv3 counts on gfx950 -- no counter sees HBM behind
    # the MALL, so the simulator's DRAM accesses (after its MALL) have no
    # hardware counterpart and are not correlated
    CorrelStat("L2->fabric read requests", r"L2_to_mem_read_requests\s*=\s*(.*)", _hw("TCC_EA0_RDREQ_sum"),
               "dram-reads"),
    CorrelStat("L2->fabric write requests", r"L2_to_mem_write_requests\s*=\s*(.*)", _hw("TCC_EA0_WRREQ_sum"),
               "dram-writes"),
    # the vector L1's requests to the L2 (the TCP->TCC counters), from the
    # matching simulator counters: icnt_total_pkts_simt_to_mem also carries
    # the instruction-fetch and scalar-cache traffic, which on CDNA leaves
    # the CU through the SQC, not the TCP
    CorrelStat("Interconnect packets SM->memory", "l1_to_l2_reqs",
               _hw("TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum", "TCP_TCC_ATOMIC_WITH_RET_REQ_sum"), "icnt-pkts",
               sim_stats=(S_L1 % ("GLOBAL_ACC_R", "MISS"), S_L2 % ("GLOBAL_ACC_W", "TOTAL_ACCESS"),
                          S_L2 % ("GLOBAL_ATOMIC", "TOTAL_ACCESS")),
               sim_eval=lambda d: sum(d.values())),
    # ---- round 3: instruction mix by the sequencer's own classes (the
    # simulator classifies each issued instruction like SQ_INSTS_*, see
    # csrc/model/sm.h sq_class / isatrace/verify.py classify) ----
    CorrelStat("VALU instructions (incl. MFMA)", S_VALU, _hw("SQ_INSTS_VALU_sum"), "valu"),
    CorrelStat("SALU instructions", S_SALU, _hw("SQ_INSTS_SALU_sum"), "salu"),
    CorrelStat("SMEM instructions", S_SMEM, _hw("SQ_INSTS_SMEM_sum"), "smem"),
    CorrelStat("VMEM read instructions", S_VMRD, _hw("SQ_INSTS_VMEM_RD_sum"), "vmem-rd"),
    CorrelStat("VMEM write instructions", S_VMWR, _hw("SQ_INSTS_VMEM_WR_sum"), "vmem-wr"),
    CorrelStat("LDS instructions", S_LDSI, _hw("SQ_INSTS_LDS_sum"), "lds-insn"),
    # ---- below the L2: Infinity Fabric traffic in 32 B sectors (TCC->EA
    # requests are 32/64/128 B), L2 dirty write-backs, L2 requests ----
    CorrelStat("L2->memory read sectors", r"L2_to_mem_read_sectors\s*=\s*(.*)", _ea_rd_sectors, "l2-mem-rd"),
    CorrelStat("L2->memory write sectors", r"L2_to_mem_write_sectors\s*=\s*(.*)",
               _hw("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"), "l2-mem-wr"),
    CorrelStat("L2 dirty write-backs", r"L2_cache_dirty_evictions\s*=\s*(.*)", _hw("TCC_WRITEBACK_sum"),
               "l2-writebacks"),
    CorrelStat("L2 requests", r"L2_total_cache_accesses\s*=\s*(.*)", _hw("TCC_REQ_sum"), "l2-req"),
    # mean L1-miss round trip (TCP->TCC read latency), shader cycles
    CorrelStat("Mean L1 miss latency", r"L1_miss_avg_latency\s*=\s*(.*)",
               _hw_ratio(("TCP_TCC_READ_REQ_LATENCY_sum",), ("TCP_TCC_READ_REQ_sum",)), "l1-miss-lat",
               ratio=True, log=False),
    # instruction cache (SQC, shared by a CU pair on CDNA4)
    CorrelStat("Instruction cache misses", r"\s+L1I_total_cache_misses\s*=\s*(.*)", _hw("SQC_ICACHE_MISSES_sum"),
               "icache-miss"),
    CorrelStat("Instruction cache accesses", r"\s+L1I_total_cache_accesses\s*=\s*(.*)",
               _hw("SQC_ICACHE_HITS_sum", "SQC_ICACHE_MISSES_sum"), "icache-acc"),
]

# rocprofv3 counter passes covering CORREL_STATS within one pass's hardware
# limits (<= 8 SQ, <= 4 TCC, <= 4 TCP counters per run)
COUNTER_GROUPS: List[str] = [
    "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR",
    "SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,TCP_TOTAL_CACHE_ACCESSES,TCP_TCC_READ_REQ,TCP_TCC_WRITE_REQ,"
    "TCP_TCC_ATOMIC_WITH_RET_REQ,TCC_HIT,TCC_MISS",
    "TCC_READ,TCC_WRITE,TCC_ATOMIC,TCC_EA0_RDREQ",
    "TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B,TCC_WRITEBACK,TCC_REQ,TCP_TCC_READ_REQ_LATENCY",
    "TCC_EA0_RDREQ_32B,TCC_EA0_RDREQ_64B,TCC_EA0_RDREQ_128B",
    "SQC_ICACHE_HITS,SQC_ICACHE_MISSES",
]


# --------------------------------------------------------------------------- HW
def _norm_kernel(name: str) -> str:
    n = name.strip().strip('"')
    n = re.sub(r"\s*\[clone .*\]$", "", n)
    return n.split("(")[0].split("<")[0].strip()


def load_hw_rocprof(hw_dir: str, burn: int = 0) -> Dict[str, List[Dict[str, List[float]]]]:
    """{app/args: [kernel_0 {col: [values over runs]}, kernel_1 ...]} from
    ``<hw_dir>/<app>/<args>/run_<i>/**/*kernel_trace.csv``."""
    out: Dict[str, List[Dict[str, List[float]]]] = {}
    for args_dir in sorted(glob.glob(os.path.join(hw_dir, "*", "*"))):
        if not os.path.isdir(args_dir):
            continue
        app = f"{os.path.basename(os.path.dirname(args_dir))}/{os.path.basename(args_dir)}"
        runs = sorted(glob.glob(os.path.join(args_dir, "run_*")), key=lambda p: int(p.rsplit("_", 1)[1]))[burn:]
        kernels: List[Dict[str, List[float]]] = []
        for r in runs:
            rows = []
            for f in glob.glob(os.path.join(r, "**", "*kernel_trace.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        try:
                            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                        except (KeyError, ValueError):
                            continue
                        name = row.get("Kernel_Name", "")
                        # runtime-internal blits (hipMemcpy/hipMemset kernels) are not application kernels
                        if "__amd_rocclr_" in name:
                            continue
                        rows.append((t0, t1, name))
            rows.sort()
            counters = _load_counters(r)
            for i, (t0, t1, name) in enumerate(rows):
                while len(kernels) <= i:
                    kernels.append(defaultdict(list))
                kernels[i]["duration_ns"].append(float(t1 - t0))
                kernels[i]["name"] = [_norm_kernel(name)]  # type: ignore[list-item]
                for k, v in (counters[i] if i < len(counters) else {}).items():
                    kernels[i][k].append(v)
        # separate counter passes (run_hw.py -c / --counter_groups): one
        # directory per (group, repeat), kernels matched by dispatch order
        for cdir in sorted(glob.glob(os.path.join(args_dir, "*"))):
            if not re.fullmatch(r"(counters|ctr\d+)_\d+", os.path.basename(cdir)):
                continue
            for i, cv in enumerate(_load_counters(cdir)):
                while len(kernels) <= i:
                    kernels.append(defaultdict(list))
                for k, v in cv.items():
                    kernels[i][k].append(v)
        if kernels:
            out[app] = [dict(k) for k in kernels]
    return out


def _load_counters(run_dir: str) -> List[Dict[str, float]]:
    """Per-dispatch counter values from rocprofv3 ``*counter_collection.csv``
    (dimension instances summed; runtime blit kernels skipped)."""
    per: Dict[int, Dict[str, float]] = {}
    for f in glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "__amd_rocclr_" in row.get("Kernel_Name", ""):
                    continue
                try:
                    d = int(row["Dispatch_Id"])
                    per.setdefault(d, {})[row["Counter_Name"] + "_sum"] = \
                        per.get(d, {}).get(row["Counter_Name"] + "_sum", 0.0) + float(row["Counter_Value"])
                except (KeyError, ValueError):
                    continue
    return [per[k] for k in sorted(per)]


def load_hw_flat(path: str) -> Dict[str, List[Dict[str, List[float]]]]:
    """Flat CSV: app,args,kernel,instance,<stat columns> (one row per run)."""
    tmp: Dict[str, Dict[int, Dict[str, List[float]]]] = defaultdict(dict)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            key = f"{row['app']}/{row['args']}"
            i = int(row.get("instance", 0))
            k = tmp[key].setdefault(i, defaultdict(list))
            k["name"] = [_norm_kernel(row.get("kernel", ""))]
            for c, v in row.items():
                if c in ("app", "args", "kernel", "instance"):
                    continue
                try:
                    k[c].append(float(v))
                except (TypeError, ValueError):
                    pass
    return {a: [dict(d[i]) for i in sorted(d)] for a, d in tmp.items()}


# -------------------------------------------------------------------------- SIM
def load_sim(csv_path: str) -> Tuple[Dict[str, Dict[str, Dict[str, List[float]]]], List[str]]:
    """{stat: {config: {app/args: [per-kernel values in launch order]}}}, configs."""
    blocks = get_stats.parse_csv_blocks(open(csv_path).read())
    out: Dict[str, Dict[str, Dict[str, List[float]]]] = {}
    configs: List[str] = []
    for stat, rows in blocks.items():
        per_cfg: Dict[str, Dict[str, List[Tuple[int, float]]]] = defaultdict(lambda: defaultdict(list))
        for order, (row, vals) in enumerate(rows.items()):
            app = row.split("--")[0]
            for cfg, v in vals.items():
                if cfg not in configs:
                    configs.append(cfg)
                try:
                    per_cfg[cfg][app].append((order, float(v)))
                except (TypeError, ValueError):
                    pass
        out[stat] = {c: {a: [v for _, v in sorted(lst)] for a, lst in apps.items()} for c, apps in per_cfg.items()}
    return out, configs


# ------------------------------------------------------------------------ stats
def error_metrics(hw: Sequence[float], sim: Sequence[float]) -> Dict[str, float]:
    h, s = np.asarray(hw, np.float64), np.asarray(sim, np.float64)
    ok = (h > 0) & np.isfinite(h) & np.isfinite(s)
    h, s = h[ok], s[ok]
    if len(h) == 0:
        return dict(n=0)
    err = (s - h) / h * 100.0
    r = dict(n=int(len(h)), mae=float(np.mean(np.abs(err))), mean_err=float(np.mean(err)),
             agg_err=float(np.sum(np.abs(s - h)) / np.sum(h) * 100.0),
             nrmse=float(np.sqrt(np.mean((s - h) ** 2)) / np.mean(h)),
             rpd=float(np.mean(np.abs(s - h) / ((s + h) / 2)) * 100.0))
    r["correl"] = float(np.corrcoef(h, s)[0, 1]) if len(h) > 1 and np.std(h) > 0 and np.std(s) > 0 else float("nan")
    return r


def _finite_mean(v) -> float:
    f = [x for x in v if math.isfinite(x)]
    return float(np.mean(f)) if f else float("nan")


def _sim_series(sim, st: CorrelStat, cfg: str) -> Dict[str, List[float]]:
    """{app: per-kernel simulator values} of one stat (derived stats evaluated
    kernel by kernel from their input stats)."""
    if st.sim_eval is None:
        return sim[st.sim_stat].get(cfg, {})
    per = [sim[s].get(cfg, {}) for s in st.sim_stats]
    out: Dict[str, List[float]] = {}
    for app in per[0]:
        if not all(app in p for p in per):
            continue
        n = min(len(p[app]) for p in per)
        vals = []
        for i in range(n):
            try:
                vals.append(float(st.sim_eval({s: p[app][i] for s, p in zip(st.sim_stats, per)})))
            except ZeroDivisionError:
                vals.append(float("nan"))
        out[app] = vals
    return out


def correlate(sim_csv: str, hw: Dict[str, List[Dict[str, List[float]]]], clock_mhz: float,
              stats: Sequence[CorrelStat] = CORREL_STATS, blacklist: Sequence[str] = (),
              hw_err_tolerance: float = 30.0, err_threshold: float = 9e9) -> Dict:
    sim, configs = load_sim(sim_csv)
    bl = [re.compile(b) for b in blacklist if b.strip()]
    result = OrderedDict()
    for st in stats:
        if st.sim_eval is None and st.sim_stat not in sim:
            continue
        if st.sim_eval is not None and any(s not in sim for s in st.sim_stats):
            continue
        agg = _finite_mean if st.ratio else (lambda v: float(np.nansum(v)))
        per_cfg = OrderedDict()
        for cfg in configs:
            apps = _sim_series(sim, st, cfg)
            app_pts, app_all, k_pts = [], [], []
            for app, svals in apps.items():
                if app not in hw or any(b.search(app) for b in bl):
                    continue
                hk = hw[app]
                n = min(len(hk), len(svals))
                if n == 0:
                    continue
                hv = [st.hw_eval(hk[i], clock_mhz) for i in range(n)]
                sv = [svals[i] * st.sim_scale for i in range(n)]
                # HW variability check (coefficient of variation over runs, %)
                spread = [np.std(hk[i]["duration_ns"]) / max(1e-9, np.mean(hk[i]["duration_ns"])) * 100
                          for i in range(n) if "duration_ns" in hk[i] and len(hk[i]["duration_ns"]) > 1]
                noisy = bool(spread) and max(spread) > hw_err_tolerance
                for i in range(n):
                    if math.isfinite(hv[i]) and hv[i] > st.drop_hw_below:
                        k_pts.append((hv[i], sv[i], f"{app}--{i}"))
                ha, sa = agg(hv), agg(sv)
                if math.isfinite(ha) and ha > st.drop_hw_below:
                    app_all.append((ha, sa, app))
                if math.isfinite(ha) and ha > st.drop_hw_below and not noisy:
                    if abs(sa - ha) / ha * 100 <= err_threshold:
                        app_pts.append((ha, sa, app))
            per_cfg[cfg] = dict(apps=app_pts, kernels=k_pts, apps_all=app_all,
                                app_metrics=error_metrics([p[0] for p in app_pts], [p[1] for p in app_pts]),
                                app_all_metrics=error_metrics([p[0] for p in app_all], [p[1] for p in app_all]),
                                kernel_metrics=error_metrics([p[0] for p in k_pts], [p[1] for p in k_pts]))
        result[st.chart_name] = dict(stat=st, configs=per_cfg)
    return result


def write_outputs(res: Dict, out_dir: str, plotname: str = "correl") -> List[str]:
    os.makedirs(out_dir, exist_ok=True)
    files, summary = [], {}
    for chart, d in res.items():
        st: CorrelStat = d["stat"]
        series = {cfg: v["apps"] for cfg, v in d["configs"].items()}
        body = [f"<h2>{chart}</h2>"]
        for cfg, v in d["configs"].items():
            m = v["app_metrics"]
            if m.get("n"):
                body.append(f"<p><b>{cfg}</b>: {m['n']} apps, MAE {m['mae']:.2f}%, aggregate error "
                            f"{m['agg_err']:.2f}%, correl {m['correl']:.4f}, NRMSE {m['nrmse']:.4f}</p>")
            summary.setdefault(chart, {})[cfg] = dict(
                app=v["app_metrics"], kernel=v["kernel_metrics"],
                # every app, including those whose HW runs vary more than -t (the
                # reference drops those from its headline, plot-correlation.py:66-90)
                app_incl_noisy=v.get("app_all_metrics", {}),
                points={a: {"hw": h, "sim": s_} for h, s_, a in v.get("apps_all", [])})
        body.append(svg.scatter(series, f"{chart}: simulation vs hardware (per app)", f"hardware {chart}",
                                f"simulated {chart}", log=st.log))
        kseries = {cfg: v["kernels"] for cfg, v in d["configs"].items()}
        body.append(svg.scatter(kseries, f"{chart}: per kernel", f"hardware {chart}", f"simulated {chart}",
                                log=st.log))
        p = os.path.join(out_dir, f"{plotname}-{st.plotfile}.html")
        with open(p, "w") as f:
            f.write(svg.page(chart, body))
        files.append(p)
    p = os.path.join(out_dir, f"{plotname}-summary.json")
    with open(p, "w") as f:
        json.dump(summary, f, indent=1)
    files.append(p)
    return files


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-c", "--csv_file", required=True, help="get_stats.py -k -K output")
    ap.add_argument("-H", "--hardware_dir", default="", help="hw_stats output directory (rocprofv3 runs)")
    ap.add_argument("-F", "--hardware_csv", default="", help="flat hardware CSV instead of -H")
    ap.add_argument("-d", "--data_mappings", default="", help="python file defining CORREL_STATS")
    ap.add_argument("-B", "--cycle_runs_to_burn", type=int, default=1)
    ap.add_argument("-b", "--blacklist", default="", help="file of app regexes to exclude")
    ap.add_argument("-t", "--hw_err_tolerance", type=float, default=30.0)
    ap.add_argument("-E", "--err_calc_threadhold", type=float, default=9e9)
    ap.add_argument("--clock_mhz", type=float, default=2400.0, help="shader clock of the measured GPU")
    ap.add_argument("-p", "--plotname", default="correl")
    ap.add_argument("-o", "--out_dir", default="correl-html")
    o = ap.parse_args(argv)
    hw = load_hw_flat(o.hardware_csv) if o.hardware_csv else load_hw_rocprof(o.hardware_dir, o.cycle_runs_to_burn)
    stats = CORREL_STATS
    if o.data_mappings:
        ns: Dict = {}
        exec(compile(open(o.data_mappings).read(), o.data_mappings, "exec"), ns)  # user's own mapping file
        stats = ns.get("CORREL_STATS", stats)
    bl = open(o.blacklist).read().splitlines() if o.blacklist else []
    res = correlate(o.csv_file, hw, o.clock_mhz, stats, bl, o.hw_err_tolerance, o.err_calc_threadhold)
    for chart, d in res.items():
        for cfg, v in d["configs"].items():
            m = v["app_metrics"]
            if m.get("n"):
                print(f"{chart:28s} {cfg:24s} apps={m['n']:3d} MAE={m['mae']:7.2f}% agg_err={m['agg_err']:7.2f}% "
                      f"correl={m['correl']:.4f} nrmse={m['nrmse']:.4f}")
    for f in write_outputs(res, o.out_dir, o.plotname):
        print("wrote", f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
