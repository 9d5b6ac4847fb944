#!/usr/bin/env python3
"""AccelWattch validation micro-benchmarks on MI355X (BASELINE config #3).

The stress kernels of csrc/ubench/ub_power.hip (idle, fp32 FMA, int32 MAD,
fp64 FMA, sqrt+exp, bf16 MFMA, LDS read, HBM read) are re-expressed as
synthetic wave64 CDNA traces with the same instruction mix, occupancy and
memory pattern (shortened: power is a rate, so a few hundred loop
iterations reach the kernel's steady state).  Each trace is simulated with
the tuned MI355X configuration and the power model on; the per-component
simulated power of every kernel (the rows of the reference's
quadprog_solver.m design matrix) is fitted to the socket power amd-smi
measured while the real kernel ran (profiles/ubench_mi355x/ub_power.log).

Outputs the calibrated XML and MAPE -- in-sample and leave-one-out, the
latter being the honest number for 8 kernels.

    python -m accel_sim_framework_distributed_amd.power.mi355x_validation
"""
from __future__ import annotations

import argparse
import csv
import json
import math
import os
import sys
import tempfile
from typing import Dict, List, Optional, Tuple

import numpy as np

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from accel_sim_framework_distributed_amd import _native  # noqa: E402
from accel_sim_framework_distributed_amd.power import calibrate, report, xmlcfg  # noqa: E402
from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder  # noqa: E402
from accel_sim_framework_distributed_amd.tracegen.format import write_kernel_binary, write_kernelslist  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TUNED = os.path.join(REPO, "configs", "tuned", "AMD_Instinct_MI355X")
MEASURED = os.path.join(REPO, "profiles", "ubench_mi355x", "ub_power.log")

CUS, BLOCK = 256, 256


def _kernel(name: str, body, iters: int, cta_per_cu: int = 8, shmem: int = 0) -> KernelBuilder:
    k = KernelBuilder(name, (CUS * cta_per_cu, 1, 1), (BLOCK, 1, 1), shmem=shmem, nregs=32, binary_version=950,
                      warp_size=64)
    k.op("v_mad_u32_u24", [1], [0])
    for i in range(iters):
        body(k, i)
    k.op("s_endpgm")
    return k


def stress_kernels(iters: int = 48) -> Dict[str, KernelBuilder]:
    """Trace builders mirroring ub_power.hip's kernels (8 independent chains each)."""
    hbm_base = 0x7F0000000000

    def fp32(k, i):
        for c in range(8):
            k.op("v_fma_f32", [8 + c], [8 + c])
        k.op("s_add_u32", [], []) if i % 8 == 7 else None

    def int32(k, i):
        for c in range(8):
            k.op("v_mul_lo_u32", [8 + c], [8 + c])
            k.op("v_add_u32", [8 + c], [8 + c])

    def fp64(k, i):
        for c in range(8):
            k.op("v_fma_f64", [8 + 2 * c], [8 + 2 * c])

    def sfu(k, i):
        k.op("v_sqrt_f32", [8], [8])
        k.op("v_exp_f32", [9], [8])
        k.op("v_add_f32", [8], [8, 9])

    def mfma(k, i):
        k.op("v_mfma_f32_32x32x16_bf16", [40], [40, 2, 3])
        k.op("v_mfma_f32_32x32x16_bf16", [56], [56, 2, 3])

    def lds(k, i):
        k.op("ds_read_b32", [8 + (i % 8)], [1], base=(i * 256) % 16384, stride=4)
        k.op("v_add_f32", [7], [7, 8 + (i % 8)])

    def hbm(k, i):
        g = k.g
        stride_cta = BLOCK * 16
        base = hbm_base + (g.cta * stride_cta + g.warp * 64 * 16 + i * (CUS * 8 * stride_cta)) % (1 << 30)
        k.op("global_load_dwordx4", [8], [1], base=base, stride=16)
        k.op("s_waitcnt")
        k.op("v_add_f32", [7], [7, 8])

    ks = {
        "fp32_fma": _kernel("k_fp32", fp32, iters),
        "int32_mad": _kernel("k_int", int32, iters),
        "fp64_fma": _kernel("k_fp64", fp64, iters),
        "sfu_sqrt_exp": _kernel("k_sfu", sfu, iters * 2),
        "mfma_bf16": _kernel("k_mfma", mfma, iters),
        "lds_read": _kernel("k_lds", lds, iters * 2, shmem=16384),
        "hbm_read": _kernel("k_hbm", hbm, iters // 2),
    }
    # idle: one tiny workgroup, the rest of the chip idle
    idle = KernelBuilder("k_idle", (1, 1, 1), (64, 1, 1), nregs=8, binary_version=950, warp_size=64)
    idle.op("s_endpgm")
    ks["idle"] = idle
    return ks


def measured_power(path: str = MEASURED) -> Dict[str, float]:
    out = {}
    with open(path) as f:
        for row in csv.reader(l for l in f if not l.startswith("#")):
            if len(row) >= 2 and row[0] and row[0] != "":
                try:
                    out[row[0]] = float(row[1])
                except ValueError:
                    pass
    return out


def measured_rows(path: str) -> Tuple[Dict[str, Dict[str, float]], Dict[str, float]]:
    """power_suite measure output: {kernel: {w, sclk, mv, temp}} in launch
    order, and the '# key value' header lines (power_cap_w, max_sclk_mhz)."""
    rows: Dict[str, Dict[str, float]] = {}
    meta: Dict[str, float] = {}

    def num(x):
        try:
            return float(x)
        except ValueError:
            return float("nan")
    with open(path) as f:
        for line in f:
            if line.startswith("#"):
                t = line[1:].split()
                if len(t) == 2:
                    meta[t[0]] = num(t[1])
                continue
            row = next(csv.reader([line]))
            if len(row) >= 2 and row[0] and not math.isnan(num(row[1])):
                rows[row[0]] = dict(w=num(row[1]), sclk=num(row[5]) if len(row) > 5 else float("nan"),
                                    mv=num(row[6]) if len(row) > 6 else float("nan"),
                                    temp=num(row[7]) if len(row) > 7 else float("nan"))
    return rows, meta


def simulate_power(work: str, xml: str, kernels: Dict[str, KernelBuilder]) -> Dict[str, Dict]:
    mod = _native.load()
    res = {}
    for name, kb in kernels.items():
        d = os.path.join(work, name)
        os.makedirs(d, exist_ok=True)
        write_kernel_binary(os.path.join(d, "kernel-1.asimk"), kb.build())
        kl = write_kernelslist(d, ["kernel-1.asimk"])
        args = ["-config", os.path.join(TUNED, "gpgpusim.config"), "-config", os.path.join(TUNED, "trace.config"),
                "-trace", kl, "-power_simulation_enabled", "1", "-accelwattch_xml_file", xml,
                "-power_report_file", os.path.join(d, "accelwattch_power_report.log"), "-gpgpu_runtime_stat", "2000:0"]
        s = mod.Simulator(args, False)
        if s.run() != 0:
            raise RuntimeError(f"{name}: simulation failed\n{s.output[-1000:]}")
        rep = report.parse_power_report(os.path.join(d, "accelwattch_power_report.log"))[0]
        res[name] = dict(report=rep, cycles=s.tot_cycle, insn=s.tot_insn)
    return res


def run(work: str, out_xml: str, iters: int = 48) -> Dict:
    base_xml = os.path.join(TUNED, "accelwattch_sass_sim.xml")
    if not os.path.exists(base_xml):
        xmlcfg.write_xml(base_xml, xmlcfg.default_params("MI355X"))
    meas = measured_power()
    ks = stress_kernels(iters)
    sim = simulate_power(work, base_xml, ks)
    names = [n for n in ks if n in meas]
    A = calibrate.design_matrix([sim[n]["report"] for n in names])
    b = np.array([meas[n] for n in names])
    before = A.sum(axis=1)
    # one factor per component group (static / VALU / special units / memory):
    # 4 parameters for 8 kernels, so leave-one-out is a real prediction
    x = calibrate.fit_groups(A, b, lower=0.05, upper=50.0)
    fit = A @ x
    loo = calibrate.leave_one_out_groups(A, b, lower=0.05, upper=50.0)
    # the per-component fit (33 free factors) for reference: exact in sample, no predictive power
    xc = calibrate.fit_scaling(A, b, lower=0.05, upper=50.0)
    calibrate.apply_factors(base_xml, out_xml, x)
    names_g, M = calibrate.group_matrix()
    summary = dict(
        kernels=names, measured_w=b.tolist(), uncalibrated_w=before.tolist(), calibrated_w=fit.tolist(),
        loo_w=loo.tolist(),
        mape_uncalibrated=calibrate.mape(before, b)[0], mape_in_sample=calibrate.mape(fit, b)[0],
        mape_leave_one_out=calibrate.mape(loo, b)[0], mae_leave_one_out_w=calibrate.mape(loo, b)[1],
        mape_per_component_in_sample=calibrate.mape(A @ xc, b)[0],
        group_factors={g: float(x[list(M[i]).index(1.0)]) if M[i].any() else 1.0 for i, g in enumerate(names_g)},
        xml=out_xml)
    return summary


SAMPLE = 250  # power sample period (core cycles) of the validation runs


def steady_components(trace_csv: str, lo: float = 0.25, hi: float = 0.75) -> Optional[Dict[str, float]]:
    """Per-component power averaged over the samples in the middle of the
    kernel (by sample index, [lo, hi)): the traced kernels are short versions
    of loops the hardware measured at steady state, so their wave-launch
    ramp and drain tail are left out.  None without enough samples."""
    if not os.path.exists(trace_csv):
        return None
    with open(trace_csv) as f:
        rows = list(csv.reader(f))
    if len(rows) < 3:
        return None
    head, data = rows[0], rows[1:]
    # the last sample is usually a partial period: drop it when there are several
    if len(data) > 3:
        data = data[:-1]
    a, b = int(len(data) * lo), max(int(len(data) * lo) + 1, int(round(len(data) * hi)))
    mid = data[a:b]
    out = {}
    for j, name in enumerate(head):
        if j < 2:
            continue
        out[name] = float(np.mean([float(r[j]) for r in mid]))
    if "STATIC_MEMP" in out:  # STATICP keeps its core (unit-mix category) part
        out["STATICP"] -= out["STATIC_MEMP"]
    return out


def simulate_trace_power_split(kernelslist: str, xml: str, work: str, config_dir: str = TUNED,
                               jobs: int = 16) -> List[Dict]:
    """simulate_trace_power with every kernel as its own CPU-engine simulation
    (bin/accel-sim.out), `jobs` at a time: the kernels are independent power
    samples, and one process per host core finishes a multi-GB trace list in
    a fraction of one sequential run."""
    import subprocess
    import threading
    import time
    from concurrent.futures import ThreadPoolExecutor
    exe = os.path.join(REPO, "bin", "accel-sim.out")
    d = os.path.dirname(os.path.abspath(kernelslist))
    kernels = [l.strip() for l in open(kernelslist) if l.strip().startswith("kernel")]
    os.makedirs(work, exist_ok=True)

    def one(i_k):
        i, k = i_k
        wd = os.path.join(work, f"k{i:03d}")
        os.makedirs(wd, exist_ok=True)
        kl = os.path.join(wd, "kernelslist.g")
        with open(kl, "w") as f:
            f.write(os.path.join(d, k) + "\n")
        rep = os.path.join(wd, "accelwattch_power_report.log")
        args = [exe, "-config", os.path.join(config_dir, "gpgpusim.config"), "-config",
                os.path.join(config_dir, "trace.config"), "-trace", kl, "-power_simulation_enabled", "1",
                "-accelwattch_xml_file", xml, "-power_report_file", rep, "-gpgpu_runtime_stat", f"{SAMPLE}:0",
                "-power_trace_enabled", "1", "-sim_engine", "cpu", "-gpgpu_kernel_launch_latency", "0",
                "-sim_first_kernel_latency", "0", "-sim_host_launch_interval", "0",
                "-sim_kernel_min_cycles_queued", "0"]
        r = subprocess.run(args, cwd=wd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                           env=dict(os.environ, OMP_NUM_THREADS="1"))
        if r.returncode != 0:
            raise RuntimeError(f"kernel {k}: simulation failed\n{r.stderr[-800:]}")
        reps = report.parse_power_report(rep)
        if len(reps) != 1:
            raise RuntimeError(f"kernel {k}: {len(reps)} power reports")
        r0 = reps[0]
        st = steady_components(os.path.join(wd, "accelwattch_power_trace.csv"))
        if st:
            r0["avg_kernel"] = r0["avg"]
            r0["avg"] = st
        return r0

    done = threading.Event()

    def beat():
        t0 = time.time()
        while not done.wait(30):
            print(f"[power validation] {len(kernels)} kernels on {jobs} cores: {time.time() - t0:.0f} s",
                  file=sys.stderr, flush=True)
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            return list(ex.map(one, enumerate(kernels)))
    finally:
        done.set()


def simulate_trace_power(kernelslist: str, xml: str, work: str, config_dir: str = TUNED,
                         engine: str = "cpu") -> List[Dict]:
    """Per-kernel power reports of one simulation of a captured trace list.
    The traced kernels are short versions of the measured loops and power is
    a rate, so the fixed kernel-launch latency (idle time) is left out."""
    mod = _native.load()
    os.makedirs(work, exist_ok=True)
    rep_path = os.path.join(work, "accelwattch_power_report.log")
    args = ["-config", os.path.join(config_dir, "gpgpusim.config"), "-config", os.path.join(config_dir, "trace.config"),
            "-trace", kernelslist, "-power_simulation_enabled", "1", "-accelwattch_xml_file", xml,
            "-power_report_file", rep_path, "-gpgpu_runtime_stat", "2000:0", "-sim_engine", engine,
            "-gpgpu_kernel_launch_latency", "0"]
    s = mod.Simulator(args, False)
    import threading
    import time
    done = threading.Event()

    def beat():  # progress line while a large trace list parses and runs
        t0 = time.time()
        while not done.wait(30):
            print(f"[power validation] simulating {kernelslist}: {time.time() - t0:.0f} s", file=sys.stderr,
                  flush=True)
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        rc = s.run()
    finally:
        done.set()
    if rc != 0:
        raise RuntimeError(f"simulation failed\n{s.output[-1000:]}")
    return report.parse_power_report(rep_path)


def run_traces(kernelslist: str, measured_csv: str, work: str, out_xml: str, config_dir: str = TUNED,
               bound: float = 20.0, engine: str = "cpu") -> Dict:
    """Validation on automatically traced kernels (bin/isatrace/power_suite
    trace) against their measured socket power (power_suite measure): the
    per-kernel component powers are fitted with one factor per FINE_GROUPS
    group, bounded to [1/bound, bound]; leave-one-out MAPE is the headline."""
    base_xml = os.path.join(config_dir, "accelwattch_sass_sim.xml")
    if not os.path.exists(base_xml):
        xmlcfg.write_xml(base_xml, xmlcfg.default_params("MI355X"))
    meas = measured_power(measured_csv)
    if engine == "cpu-split":
        reps = simulate_trace_power_split(kernelslist, base_xml, work, config_dir,
                                          int(os.environ.get("MAX_JOBS", "16") or 16))
    else:
        reps = simulate_trace_power(kernelslist, base_xml, work, config_dir, engine)
    order = list(meas)  # measure mode prints the kernels in launch order
    if len(reps) != len(order):
        raise RuntimeError(f"{len(reps)} simulated kernels vs {len(order)} measured")
    A = calibrate.design_matrix(reps, calibrate.CAL_COMPONENTS_BASE)
    b = np.array([meas[n] for n in order])
    rows, meta = measured_rows(measured_csv)
    if all(not math.isnan(rows[n]["sclk"]) for n in order) and meta.get("power_cap_w", float("nan")) > 0:
        s = fit_report_dvfs(A, b, order, [rows[n]["sclk"] for n in order], [rows[n]["mv"] for n in order],
                            meta["power_cap_w"], meta.get("max_sclk_mhz", float("nan")), bound)
        calibrate.apply_factors(base_xml, out_xml, s.pop("_x"), power_cap=s["power_cap_w"])
        _set_dvfs_params(out_xml, s)
    else:
        A = calibrate.design_matrix(reps)
        s = fit_report(A, b, order, bound)
        calibrate.apply_factors(base_xml, out_xml, s.pop("_x"), power_cap=s["power_cap_w"])
    s.update(sim_cycles=[r.get("gpu_sim_cycle", 0.0) for r in reps], traces="automatic ISA traces (isatrace)",
             xml=out_xml)
    return s


# the single-unit kernels of the power suite, at every occupancy they run at:
# the calibration set (the occupancy points separate a unit's always-on
# power from its per-instruction energy).  Every unit mix is held out.
CAL_KERNELS = ["idle", "fp32_fma", "fp32_add", "int32_add", "int32_mul", "fp64_fma", "fp64_add", "sfu_sqrt_exp",
               "mfma_bf16", "lds_read", "lds_write", "hbm_read", "hbm_write", "l2_read", "l2_write", "l1_read",
               "atomic_l2", "fp32_fma_occ1", "fp32_fma_occ2", "fp32_fma_occ4", "mfma_bf16_occ2", "mfma_bf16_occ4",
               "sfu_occ2", "fp64_fma_occ2", "hbm_read_occ2", "lds_read_occ2", "lds_write_occ2", "hbm_write_occ2",
               "int32_add_occ2", "fp32_fma_light"]


def fit_heldout(A: np.ndarray, b: np.ndarray, order: List[str], sclk: List[float], mv: List[float], cap: float,
                max_sclk: float, cal: List[str] = CAL_KERNELS, bound: float = 20.0) -> Dict:
    """Calibrate one factor per execution unit (calibrate.UNIT_GROUPS) on the
    single-unit kernels only, each kernel's components moved to its measured
    clock (DVFS matrix), then predict the disjoint held-out kernels: their
    MAPE is the headline (reference util/accelwattch: quadprog_solver.m fits
    on the validation micro-benchmarks, the suite validates)."""
    sclk = np.asarray(sclk, np.float64)
    fmax = max_sclk if max_sclk and not math.isnan(max_sclk) else float(np.nanmax(sclk))
    ratios = np.clip(sclk / fmax, 0.05, 1.0)
    v_floor = calibrate.v_floor_from_measurements(sclk, mv, fmax)
    vsrc = "measured rail voltage vs clock"
    if v_floor is None:
        v_floor, vsrc = DEFAULT_V_FLOOR, ("not measurable here: amd-smi reports no graphics rail voltage on this "
                                          "node (vddgfx NaN) and a non-root user cannot set clocks; the line's "
                                          "floor is assumed")
    ci = [i for i, n in enumerate(order) if n in cal]
    vi = [i for i, n in enumerate(order) if n not in cal]
    groups = calibrate.UNIT_GROUPS
    Ad = calibrate.dvfs_matrix(A, ratios, v_floor)
    # the issue-weighted static column may be left out entirely (factor 0:
    # the reference's residency-only static power); every other group is
    # bounded to [1 / bound, bound]
    free0 = {"static_issue"}
    lower = np.array([0.0 if g in free0 else 1.0 / bound for g in groups])
    x = calibrate.fit_groups_relative(Ad[ci], b[ci], groups=groups, lower=lower, upper=bound)
    pred = Ad @ x
    # uncalibrated: the base XML's model (the alternative static column off)
    comps = calibrate._comps(Ad.shape[1])
    before = Ad[:, [j for j, c in enumerate(comps) if c != "STATIC_ISSUEP"]].sum(axis=1)
    gf = calibrate.group_factors(x, groups)
    at_bound = [g for g, v in gf.items() if (g not in free0 and v <= 1.0 / bound * 1.001) or v >= bound * 0.999]
    # groups no calibration kernel exercises keep factor 1 (reported)
    undriven = [g for g in groups if not any(Ad[i, [comps.index(c) for c in groups[g] if c in comps]].sum() > 0
                                             for i in ci)]
    bv, pv = b[vi], pred[vi]
    return dict(kernels=list(order), calibration_kernels=[order[i] for i in ci],
                heldout_kernels=[order[i] for i in vi], measured_w=b.tolist(), uncalibrated_w=before.tolist(),
                calibrated_w=pred.tolist(),
                mape_heldout=calibrate.mape(pv, bv)[0], mae_heldout_w=calibrate.mape(pv, bv)[1],
                mape_heldout_uncalibrated=calibrate.mape(before[vi], bv)[0],
                mape_calibration_in_sample=calibrate.mape(pred[ci], b[ci])[0],
                mape_all=calibrate.mape(pred, b)[0], group_factors=gf, factors_at_bound=at_bound,
                groups_not_driven=undriven, power_cap_w=float(cap), max_sclk_mhz=float(fmax),
                measured_sclk_mhz=sclk.tolist(), measured_clock_ratio=ratios.tolist(),
                measured_vddgfx_mv=[float(v) for v in mv], v_floor=float(v_floor), v_floor_source=vsrc,
                components=list(comps), components_w=np.asarray(A).tolist(), groups=groups,
                bounds=[1.0 / bound, bound],
                model="per-unit factors fitted on single-unit kernels, validated on held-out mixes", _x=x)


def run_heldout(kernelslist: str, measured_csv: str, work: str, out_xml: str, config_dir: str = TUNED,
                bound: float = 20.0, engine: str = "cpu-split") -> Dict:
    base_xml = os.path.join(config_dir, "accelwattch_sass_sim.xml")
    if not os.path.exists(base_xml):
        xmlcfg.write_xml(base_xml, xmlcfg.default_params("MI355X"))
    meas = measured_power(measured_csv)
    if engine == "cpu-split":
        reps = simulate_trace_power_split(kernelslist, base_xml, work, config_dir,
                                          int(os.environ.get("MAX_JOBS", "16") or 16))
    else:
        reps = simulate_trace_power(kernelslist, base_xml, work, config_dir, engine)
    order = list(meas)
    if len(reps) != len(order):
        raise RuntimeError(f"{len(reps)} simulated kernels vs {len(order)} measured")
    A = calibrate.design_matrix(reps, calibrate.CAL_COMPONENTS)
    b = np.array([meas[n] for n in order])
    rows, meta = measured_rows(measured_csv)
    s = fit_heldout(A, b, order, [rows[n]["sclk"] for n in order], [rows[n]["mv"] for n in order],
                    meta.get("power_cap_w", float("nan")), meta.get("max_sclk_mhz", float("nan")), bound=bound)
    calibrate.apply_factors(base_xml, out_xml, s.pop("_x"), power_cap=s["power_cap_w"])
    _set_dvfs_params(out_xml, dict(v_floor=s["v_floor"], dvfs_min_clock_ratio=max(
        0.3, min(1.0, float(np.nanmin(s["measured_clock_ratio"])) * 0.9))))
    s.update(sim_cycles=[r.get("gpu_sim_cycle", 0.0) for r in reps], traces="automatic ISA traces (isatrace)",
             xml=out_xml)
    return s


def _set_dvfs_params(xml: str, s: Dict) -> None:
    p = xmlcfg.read_xml(xml)
    p["dvfs_v_floor"] = float(s["v_floor"])
    p["dvfs_min_clock_ratio"] = float(s["dvfs_min_clock_ratio"])
    xmlcfg.write_xml(xml, p, comment="calibrated with measured clocks; power_cap measured by amd-smi")


DEFAULT_V_FLOOR = 0.6


def fit_report_dvfs(A: np.ndarray, b: np.ndarray, order: List[str], sclk: List[float], mv: List[float],
                    cap: float, max_sclk: float, bound: float = 20.0, v_floor: Optional[float] = None) -> Dict:
    """Validation with the DVFS model and MEASURED inputs only: the package
    power limit and every kernel's graphics clock come from amd-smi
    (power_suite measure); V(f) from the measured rail voltages when the
    firmware reports them.  The FINE_GROUPS factors are fitted on relative
    error with each kernel's components moved to its measured clock;
    leave-one-out predicts the held-out kernel both at its measured clock
    (the headline, like AccelWattch's validation with measured voltage) and
    fully predictively, at the clock the governor picks under the cap."""
    sclk = np.asarray(sclk, np.float64)
    fmax = max_sclk if max_sclk and not math.isnan(max_sclk) else float(np.nanmax(sclk))
    ratios = np.clip(sclk / fmax, 0.05, 1.0)
    vsrc = "given"
    if v_floor is None:
        v_floor = calibrate.v_floor_from_measurements(sclk, mv, fmax)
        vsrc = "measured rail voltage vs clock"
        if v_floor is None:
            v_floor, vsrc = DEFAULT_V_FLOOR, "assumed (no rail voltage reported by amd-smi)"
    s_min = float(max(0.3, min(1.0, np.nanmin(ratios) * 0.9)))
    split = A.shape[1] in (len(calibrate.CAL_COMPONENTS), len(calibrate.CAL_COMPONENTS_BASE))
    groups = calibrate.POWER_GROUPS if split else calibrate.FINE_GROUPS
    kw = dict(groups=groups, lower=1.0 / bound, upper=bound)
    Ad = calibrate.dvfs_matrix(A, ratios, v_floor)
    x = calibrate.fit_groups_relative(Ad, b, **kw)
    fit = Ad @ x
    loo_meas, loo_gov, s_gov = calibrate.leave_one_out_dvfs(A, b, ratios, v_floor, cap, s_min, **kw)
    gov_fit = np.array([calibrate.governor_ratio(A[i], x, cap, v_floor, s_min) for i in range(len(b))])
    gf = calibrate.group_factors(x, groups)
    at_bound = [g for g, v in gf.items() if v <= 1.0 / bound * 1.001 or v >= bound * 0.999]
    before = A.sum(axis=1)
    return dict(kernels=list(order), measured_w=b.tolist(), uncalibrated_w=before.tolist(), calibrated_w=fit.tolist(),
                loo_w=loo_meas.tolist(), mape_uncalibrated=calibrate.mape(before, b)[0],
                mape_in_sample=calibrate.mape(fit, b)[0], mape_leave_one_out=calibrate.mape(loo_meas, b)[0],
                mae_leave_one_out_w=calibrate.mape(loo_meas, b)[1], group_factors=gf, factors_at_bound=at_bound,
                power_cap_w=float(cap), power_cap_source="measured (amd-smi power cap)", max_sclk_mhz=float(fmax),
                measured_sclk_mhz=sclk.tolist(), measured_clock_ratio=ratios.tolist(),
                measured_vddgfx_mv=[float(v) for v in mv], v_floor=float(v_floor), v_floor_source=vsrc,
                dvfs_min_clock_ratio=s_min,
                governor=dict(loo_w=loo_gov.tolist(), mape_leave_one_out=calibrate.mape(loo_gov, b)[0],
                              loo_clock_ratio=s_gov.tolist(), fit_clock_ratio=gov_fit.tolist(),
                              clock_ratio_mae=float(np.mean(np.abs(s_gov - ratios))),
                              throttled_kernels=[n for n, r in zip(order, ratios) if r < 0.98]),
                components=calibrate._comps(A.shape[1]), components_w=np.asarray(A).tolist(), groups=groups,
                bounds=[1.0 / bound, bound], model="DVFS: measured cap and clocks, V(f) line", _x=x)


def fit_report(A: np.ndarray, b: np.ndarray, order: List[str], bound: float = 20.0) -> Dict:
    """Fit the FINE_GROUPS factors plus the package power cap to measured
    power (rows of A: per-kernel simulated component powers with no cap in
    the XML) and score it in-sample and leave-one-out.  The uncapped linear
    fit is reported alongside for comparison."""
    before = A.sum(axis=1)
    kw = dict(groups=calibrate.FINE_GROUPS, lower=1.0 / bound, upper=bound)
    x, cap = calibrate.fit_groups_capped(A, b, **kw)
    loo = calibrate.leave_one_out_capped(A, b, **kw)
    fit = calibrate.predict_capped(A, x, cap)
    x_lin = calibrate.fit_groups(A, b, **kw)
    loo_lin = calibrate.leave_one_out_groups(A, b, **kw)
    gf = calibrate.group_factors(x, calibrate.FINE_GROUPS)
    at_bound = [g for g, v in gf.items() if v <= 1.0 / bound * 1.001 or v >= bound * 0.999]
    return dict(kernels=list(order), measured_w=b.tolist(), uncalibrated_w=before.tolist(), calibrated_w=fit.tolist(),
                loo_w=loo.tolist(), mape_uncalibrated=calibrate.mape(before, b)[0],
                mape_in_sample=calibrate.mape(fit, b)[0], mape_leave_one_out=calibrate.mape(loo, b)[0],
                mae_leave_one_out_w=calibrate.mape(loo, b)[1], group_factors=gf, factors_at_bound=at_bound,
                power_cap_w=cap, capped_kernels=[n for n, v in zip(order, A @ x) if v > cap],
                linear_no_cap=dict(mape_in_sample=calibrate.mape(A @ x_lin, b)[0],
                                   mape_leave_one_out=calibrate.mape(loo_lin, b)[0],
                                   group_factors=calibrate.group_factors(x_lin, calibrate.FINE_GROUPS)),
                components=list(calibrate.COMPONENTS), components_w=np.asarray(A).tolist(), bounds=[1.0 / bound, bound],
                _x=x)


def refit(json_path: str, out_xml: str, config_dir: str = TUNED, bound: float = 20.0) -> Dict:
    """Re-run the fit on a saved validation record (its per-kernel component
    powers and measured watts) without re-simulating."""
    with open(json_path) as f:
        old = json.load(f)
    A = np.asarray(old["components_w"], np.float64)
    b = np.asarray(old["measured_w"], np.float64)
    base_xml = os.path.join(config_dir, "accelwattch_sass_sim.xml")
    if "calibration_kernels" in old:
        s = fit_heldout(A, b, old["kernels"], old["measured_sclk_mhz"], old.get("measured_vddgfx_mv", []),
                        old["power_cap_w"], old.get("max_sclk_mhz", float("nan")), bound=bound)
        calibrate.apply_factors(base_xml, out_xml, s.pop("_x"), power_cap=s["power_cap_w"])
    elif "measured_sclk_mhz" in old:
        s = fit_report_dvfs(A, b, old["kernels"], old["measured_sclk_mhz"], old.get("measured_vddgfx_mv", []),
                            old["power_cap_w"], old.get("max_sclk_mhz", float("nan")), bound)
        calibrate.apply_factors(base_xml, out_xml, s.pop("_x"), power_cap=s["power_cap_w"])
        _set_dvfs_params(out_xml, s)
    else:
        s = fit_report(A, b, old["kernels"], bound)
        calibrate.apply_factors(base_xml, out_xml, s.pop("_x"), power_cap=s["power_cap_w"])
    for k in ("sim_cycles", "traces", "note"):
        if k in old:
            s[k] = old[k]
    s["xml"] = os.path.relpath(out_xml, REPO) if out_xml.startswith(REPO) else out_xml
    return s


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-o", "--out_xml", default=os.path.join(TUNED, "accelwattch_sass_sim_calibrated.xml"))
    ap.add_argument("-j", "--json", default=os.path.join(REPO, "profiles", "power_mi355x_validation.json"))
    ap.add_argument("-w", "--work", default="")
    ap.add_argument("-t", "--traces", default="", help="kernelslist.g of bin/isatrace/power_suite trace")
    ap.add_argument("-m", "--measured", default="", help="CSV of power_suite measure")
    ap.add_argument("-c", "--config_dir", default=TUNED)
    ap.add_argument("-e", "--engine", default="cpu", help="cpu | gpu (the MI355X cycle engine)")
    ap.add_argument("--refit", default="", help="re-fit a saved validation JSON (no simulation)")
    ap.add_argument("--heldout", action="store_true",
                    help="calibrate on the single-unit kernels, validate on the held-out rest")
    o = ap.parse_args(argv)
    work = o.work or tempfile.mkdtemp(prefix="asim_power_")
    if o.refit:
        s = refit(o.refit, o.out_xml, o.config_dir)
    elif o.traces and o.heldout:
        s = run_heldout(o.traces, o.measured or MEASURED, work, o.out_xml, o.config_dir, engine=o.engine)
    if "calibration_kernels" in s:  # held-out record (run_heldout, or a refit of one)
        with open(o.json, "w") as f:
            json.dump(s, f, indent=1)
        print(f"{'kernel':16s} {'set':4s} {'measured':>9s} {'uncal':>9s} {'model':>9s}")
        for i, n in enumerate(s["kernels"]):
            print(f"{n:16s} {'cal' if n in s['calibration_kernels'] else 'val':4s} {s['measured_w'][i]:9.1f} "
                  f"{s['uncalibrated_w'][i]:9.1f} {s['calibrated_w'][i]:9.1f}")
        print(f"held-out MAPE {s['mape_heldout']:.2f}% ({s['mae_heldout_w']:.1f} W) on {len(s['heldout_kernels'])} "
              f"kernels; uncalibrated {s['mape_heldout_uncalibrated']:.2f}%; calibration in-sample "
              f"{s['mape_calibration_in_sample']:.2f}% on {len(s['calibration_kernels'])}")
        print("group factors:", {g: round(v, 3) for g, v in s["group_factors"].items()}, "at bound:",
              s["factors_at_bound"], "not driven:", s["groups_not_driven"])
        return 0
    if o.refit:
        pass
    elif o.traces:
        s = run_traces(o.traces, o.measured or MEASURED, work, o.out_xml, o.config_dir, engine=o.engine)
    else:
        s = run(work, o.out_xml)
    with open(o.json, "w") as f:
        json.dump(s, f, indent=1)
    print(f"{'kernel':14s} {'measured':>9s} {'uncal':>9s} {'fit':>9s} {'LOO':>9s}")
    for i, n in enumerate(s["kernels"]):
        print(f"{n:14s} {s['measured_w'][i]:9.1f} {s['uncalibrated_w'][i]:9.1f} {s['calibrated_w'][i]:9.1f} "
              f"{s['loo_w'][i]:9.1f}")
    print(f"MAPE uncalibrated {s['mape_uncalibrated']:.2f}%  in-sample {s['mape_in_sample']:.2f}%  "
          f"leave-one-out {s['mape_leave_one_out']:.2f}% ({s['mae_leave_one_out_w']:.1f} W)")
    print("group factors:", {g: round(v, 3) for g, v in s["group_factors"].items()},
          "at bound:", s.get("factors_at_bound"), "power cap:", s.get("power_cap_w"))
    if "governor" in s:
        g = s["governor"]
        print(f"DVFS: measured cap {s['power_cap_w']:.0f} W, v_floor {s['v_floor']:.3f} ({s['v_floor_source']}); "
              f"governor-predicted LOO MAPE {g['mape_leave_one_out']:.2f}%, clock-ratio MAE {g['clock_ratio_mae']:.3f}, "
              f"throttled: {g['throttled_kernels']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
