"""Calibrate AccelWattch scaling factors against measured power.

Same formulation as the reference's util/accelwattch/quadprog_solver.m:30-92
(solved there with MATLAB ``lsqlin``): rows are kernels, columns the
simulated per-component average power at the current scaling factors, ``b``
the measured hardware power; find multiplicative corrections ``x`` with
``lower <= x <= upper`` and optional ordering constraints ``C x <= d``
("an INT op costs no more than an FP op" ...) minimising ``||A x - b||^2``.
Solved with scipy (bounded least squares, or SLSQP when constraints are
given).  ``apply_factors`` folds ``x`` back into an XML.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .report import COMPONENTS
from .xmlcfg import read_xml, write_xml

# report component -> XML parameters it scales
COMPONENT_PARAMS: Dict[str, List[str]] = {
    "IBP": ["TOT_INST"], "ICP": ["IC_H", "IC_M"], "DCP": ["DC_RH", "DC_RM", "DC_WH", "DC_WM"], "TCP": [],
    "CCP": ["CC_H", "CC_M"], "SHRDP": ["SHRD_ACC"], "RFP": ["REG_RD", "REG_WR"], "INTP": ["INT_ACC"],
    "FPUP": ["FP_ACC"], "DPUP": ["DP_ACC"], "INT_MUL24P": [], "INT_MUL32P": [], "INT_MULP": ["INT_MUL_ACC"],
    "INT_DIVP": [], "FP_MULP": ["FP_MUL_ACC"], "FP_DIVP": [], "FP_SQRTP": ["FP_SQRT_ACC"], "FP_LGP": ["FP_LG_ACC"],
    "FP_SINP": ["FP_SIN_ACC"], "FP_EXP": ["FP_EXP_ACC"], "DP_MULP": ["DP_MUL_ACC"], "DP_DIVP": [],
    "TENSORP": ["TENSOR_ACC"], "TEXP": ["TEX_ACC"], "SCHEDP": ["FP_INT"], "L2CP": ["L2_RH", "L2_RM", "L2_WH", "L2_WM"],
    "MCP": ["MEM_PRE"], "NOCP": ["NOC_A"], "DRAMP": ["MEM_RD", "MEM_WR"], "PIPEP": ["PIPE_A"],
    "IDLE_COREP": ["idle_core_power"], "CONSTP": ["constant_power"], "STATICP": None,  # None: every static_* param
    # calibration-only column: the LDS / L1 / L2 "unit in use" part of STATICP
    # (power trace column STATIC_MEMP); with it, STATICP is the core part
    "STATIC_MEMP": ["static_shared_flane", "static_l1_flane", "static_l2_flane"],
    # calibration-only column: the core static power weighted by instruction
    # issue instead of residency (power trace column STATIC_ISSUEP); its
    # factor and STATICP's set the XML's static scale and static_issue_weight
    "STATIC_ISSUEP": [],
}
# the components of the DVFS-aware calibration: the report's, with STATICP
# split into core and memory-unit static power
CAL_COMPONENTS: List[str] = list(COMPONENTS) + ["STATIC_MEMP", "STATIC_ISSUEP"]
# without the issue-weighted alternative (fits whose groups do not choose
# between the two static columns)
CAL_COMPONENTS_BASE: List[str] = list(COMPONENTS) + ["STATIC_MEMP"]


def _comps(n: int) -> List[str]:
    """The component list a row / factor vector of length n refers to (records
    from before the issue-weighted column have one calibration column)."""
    if n == len(CAL_COMPONENTS):
        return CAL_COMPONENTS
    if n == len(COMPONENTS) + 1:
        return list(COMPONENTS) + ["STATIC_MEMP"]
    return list(COMPONENTS)


def design_matrix(kernels: Sequence[Dict], components: Sequence[str] = COMPONENTS) -> np.ndarray:
    return np.array([[k["avg"].get(c, 0.0) for c in components] for k in kernels], dtype=np.float64)


def fit_scaling(A: np.ndarray, b: np.ndarray, lower: float | np.ndarray = 0.1, upper: float | np.ndarray = 1000.0,
                C: Optional[np.ndarray] = None, d: Optional[np.ndarray] = None,
                fixed: Optional[Iterable[int]] = None) -> np.ndarray:
    """x >= 0 minimising ||A x - b||^2 with bounds and C x <= d.  Columns that
    are identically zero (component never active) keep x = 1, as do ``fixed``."""
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    n = A.shape[1]
    lo = np.broadcast_to(np.asarray(lower, np.float64), (n,)).copy()
    hi = np.broadcast_to(np.asarray(upper, np.float64), (n,)).copy()
    free = np.abs(A).sum(axis=0) > 0
    for i in fixed or ():
        free[i] = False
    x = np.ones(n)
    idx = np.flatnonzero(free)
    if len(idx) == 0:
        return x
    # account for the fixed columns at x = 1
    b_eff = b - A[:, ~free].sum(axis=1)
    Af = A[:, idx]
    # column scaling keeps the problem well conditioned (powers span 0.01..100 W)
    scale = np.linalg.norm(Af, axis=0)
    scale[scale == 0] = 1.0
    As = Af / scale
    lo_s, hi_s = lo[idx] * scale, hi[idx] * scale
    if C is None:
        from scipy.optimize import lsq_linear
        r = lsq_linear(As, b_eff, bounds=(lo_s, hi_s), method="bvls", lsmr_tol="auto")
        x[idx] = r.x / scale
        return x
    from scipy.optimize import minimize
    C = np.asarray(C, np.float64)
    d = np.asarray(d, np.float64) - C[:, ~free].sum(axis=1)
    Cs = C[:, idx] / scale

    def f(z):
        r = As @ z - b_eff
        return 0.5 * float(r @ r), As.T @ r

    z0 = np.clip(scale, lo_s, hi_s)
    cons = [dict(type="ineq", fun=lambda z: d - Cs @ z, jac=lambda z: -Cs)]
    r = minimize(f, z0, jac=True, bounds=list(zip(lo_s, hi_s)), constraints=cons, method="SLSQP",
                 options=dict(maxiter=500, ftol=1e-12))
    x[idx] = r.x / scale
    return x


# coarse component groups: one scaling factor per group keeps the number of
# fitted parameters well below the number of validation kernels
COMPONENT_GROUPS: Dict[str, List[str]] = {
    "idle": ["CONSTP", "IDLE_COREP"],
    "static": ["STATICP"],
    "valu": ["IBP", "ICP", "RFP", "INTP", "FPUP", "DPUP", "INT_MUL24P", "INT_MUL32P", "INT_MULP", "INT_DIVP",
             "FP_MULP", "FP_DIVP", "DP_DIVP", "SCHEDP", "PIPEP"],
    "special": ["FP_SQRTP", "FP_LGP", "FP_SINP", "FP_EXP", "DP_MULP", "TENSORP", "TEXP"],
    "memory": ["DCP", "TCP", "CCP", "SHRDP", "L2CP", "MCP", "NOCP", "DRAMP"],
}


# finer groups for the 24-kernel validation suite (csrc/apps/power_suite.hip):
# 9 factors, each exercised by several kernels (a factor only one kernel
# drives cannot be predicted leave-one-out)
FINE_GROUPS: Dict[str, List[str]] = {
    "idle_static": ["CONSTP", "IDLE_COREP", "STATICP"],
    "frontend": ["IBP", "ICP", "SCHEDP", "PIPEP", "RFP"],
    "valu": ["FPUP", "FP_MULP", "FP_DIVP", "INTP", "INT_MUL24P", "INT_MUL32P", "INT_MULP", "INT_DIVP"],
    "fp64": ["DPUP", "DP_MULP", "DP_DIVP"],
    "sfu": ["FP_SQRTP", "FP_LGP", "FP_SINP", "FP_EXP"],
    "tensor": ["TENSORP", "TEXP"],
    "lds": ["SHRDP"],
    "cache": ["DCP", "TCP", "CCP", "L2CP", "NOCP"],
    "dram": ["DRAMP", "MCP"],
}


def group_matrix(components: Sequence[str] = COMPONENTS, groups: Dict[str, List[str]] = COMPONENT_GROUPS):
    """(G x C) 0/1 matrix mapping group factors to component factors."""
    names = list(groups)
    M = np.zeros((len(names), len(components)))
    for gi, g in enumerate(names):
        for c in groups[g]:
            if c in components:
                M[gi, list(components).index(c)] = 1.0
    return names, M


def fit_groups(A: np.ndarray, b: np.ndarray, groups: Dict[str, List[str]] = COMPONENT_GROUPS, **kw) -> np.ndarray:
    """Per-component factors constrained to be equal within each group."""
    names, M = group_matrix(components=_comps(np.asarray(A).shape[1]), groups=groups)
    xg = fit_scaling(np.asarray(A) @ M.T, b, **kw)
    x = M.T @ xg
    x[M.sum(axis=0) == 0] = 1.0
    return x


def leave_one_out_groups(A: np.ndarray, b: np.ndarray, **kw) -> np.ndarray:
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    out = np.zeros(len(b))
    for i in range(len(b)):
        keep = np.arange(len(b)) != i
        out[i] = A[i] @ fit_groups(A[keep], b[keep], **kw)
    return out


def group_factors(x: Sequence[float], groups: Dict[str, List[str]] = COMPONENT_GROUPS) -> Dict[str, float]:
    names, M = group_matrix(components=_comps(len(x)), groups=groups)
    return {g: float(np.asarray(x)[list(M[i]).index(1.0)]) if M[i].any() else 1.0 for i, g in enumerate(names)}


def fit_groups_capped(A: np.ndarray, b: np.ndarray, groups: Dict[str, List[str]] = FINE_GROUPS,
                      lower: float = 0.05, upper: float = 20.0, restarts: int = 8) -> Tuple[np.ndarray, float]:
    """Group factors plus a package power cap: ``P = min(cap, A x)``.

    MI355X power management holds the socket at its limit by lowering clocks,
    so every compute-saturating kernel measures about the same power whatever
    its activity (1280-1330 W in profiles/power_mi355x_validation.json).  A
    purely linear model has to compromise between those kernels and the rest;
    with the cap the linear part is fitted where the part is not throttled.
    The objective is the relative error (MAPE is the reported metric); the
    problem is piecewise linear, so a few deterministic restarts pick the
    best local minimum.  Returns (per-component factors, cap in W)."""
    from scipy.optimize import least_squares
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    names, M = group_matrix(groups=groups)
    G = A @ M.T
    n = G.shape[1]
    active = np.abs(G).sum(axis=0) > 0

    def res(z):
        return (np.minimum(G @ z[:n], z[n]) - b) / b

    lb = np.r_[np.where(active, lower, 1.0 - 1e-9), b.max() * 0.95]
    ub = np.r_[np.where(active, upper, 1.0 + 1e-9), b.max() * 1.3]
    best = None
    for k in range(restarts):
        z0 = np.ones(n + 1)
        z0[n] = b.max() * 1.02
        if k:
            z0[:n] = np.where(active, np.exp(np.random.RandomState(k).uniform(np.log(0.2), np.log(5.0), n)), 1.0)
        r = least_squares(res, np.clip(z0, lb + 1e-9, ub - 1e-9), bounds=(lb, ub))
        if best is None or r.cost < best.cost:
            best = r
    xg = best.x[:n]
    x = M.T @ xg
    x[M.sum(axis=0) == 0] = 1.0
    return x, float(best.x[n])


def predict_capped(A: np.ndarray, x: np.ndarray, cap: float) -> np.ndarray:
    return np.minimum(np.asarray(A, np.float64) @ x, cap)


def leave_one_out_capped(A: np.ndarray, b: np.ndarray, **kw) -> np.ndarray:
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    out = np.zeros(len(b))
    for i in range(len(b)):
        keep = np.arange(len(b)) != i
        x, cap = fit_groups_capped(A[keep], b[keep], **kw)
        out[i] = predict_capped(A[i:i + 1], x, cap)[0]
    return out


def mape(pred: Sequence[float], meas: Sequence[float]) -> Tuple[float, float]:
    """(mean absolute percentage error %, mean absolute error W)."""
    p, m = np.asarray(pred, np.float64), np.asarray(meas, np.float64)
    return float(np.mean(np.abs(p - m) / np.abs(m)) * 100.0), float(np.mean(np.abs(p - m)))


def leave_one_out(A: np.ndarray, b: np.ndarray, **kw) -> np.ndarray:
    """Predictions where each kernel's power comes from a fit that excluded it."""
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    out = np.zeros(len(b))
    for i in range(len(b)):
        keep = np.arange(len(b)) != i
        x = fit_scaling(A[keep], b[keep], **kw)
        out[i] = A[i] @ x
    return out


def apply_factors(xml_in: str, xml_out: str, x: Sequence[float], components: Optional[Sequence[str]] = None,
                  power_cap: Optional[float] = None) -> Dict:
    """Multiply the XML parameters behind every component by its factor
    (and set the package ``power_cap`` when one was fitted)."""
    p = read_xml(xml_in)
    if power_cap:
        p["power_cap"] = float(power_cap)
    components = list(components) if components is not None else _comps(len(x))
    split = "STATIC_MEMP" in components
    fx = dict(zip(components, (float(v) for v in x)))
    issue = "STATIC_ISSUEP" in components and "STATICP" in components
    for c, f in zip(components, x):
        keys = COMPONENT_PARAMS.get(c)
        if keys is None:
            keys = [k for k in p if k.startswith("static_") and k != "static_issue_weight"
                    and not (split and k in COMPONENT_PARAMS["STATIC_MEMP"])]
            if issue:
                # core static = base x ((1 - w) busy + w issue); the fit scales
                # the column pair (STATICP, STATIC_ISSUEP) = (core static,
                # base x issue) by (f1, f2): base' = base (f1 + f2),
                # w' = (f1 w + f2) / (f1 + f2)
                f1, f2, w = fx["STATICP"], fx["STATIC_ISSUEP"], float(p.get("static_issue_weight", 0.0))
                f = f1 + f2
                p["static_issue_weight"] = (f1 * w + f2) / f if f > 0 else w
        for k in keys:
            p[k] = p.get(k, 1.0) * float(f)
    write_xml(xml_out, p, comment=f"calibrated from {xml_in}")
    return p


# ---- DVFS-aware calibration (round 3) ---------------------------------------
# The power model runs a kernel at core clock ratio s = f / f_nominal with the
# rail voltage V(s)/V(1) = v_floor + (1 - v_floor) s (csrc/power/power.cc):
# core dynamic power ~ s V^2, static and idle-core power ~ V, DRAM ~ s (its own
# rail), the constant term fixed.  A row of A holds a kernel's component powers
# simulated at the nominal clock; dvfs_scale() maps it to clock ratio s.
_DVFS_V = ("STATICP", "IDLE_COREP", "STATIC_MEMP", "STATIC_ISSUEP")
_DVFS_FIXED = ("CONSTP",)
_DVFS_S = ("DRAMP", "MCP")


def voltage_ratio(s, v_floor: float):
    return v_floor + (1.0 - v_floor) * np.asarray(s, np.float64)


def dvfs_scale(s: float, v_floor: float, components: Optional[Sequence[str]] = None, n: int = 0) -> np.ndarray:
    v = float(voltage_ratio(s, v_floor))
    components = components if components is not None else _comps(n or len(COMPONENTS))
    return np.array([1.0 if c in _DVFS_FIXED else v if c in _DVFS_V else s if c in _DVFS_S else s * v * v
                     for c in components])


def dvfs_matrix(A: np.ndarray, ratios: Sequence[float], v_floor: float) -> np.ndarray:
    A = np.asarray(A, np.float64)
    return np.stack([A[i] * dvfs_scale(float(r), v_floor, n=A.shape[1]) for i, r in enumerate(ratios)])


# groups of the DVFS-aware MI355X calibration: one factor per pipe the
# validation kernels exercise separately -- the always-on part, the VALU pipe
# (instruction issue, fp32 / int / fp64 / transcendental work), the matrix
# cores, the memory pipeline on the CU and in the L2 (LDS, L1, L2, NoC and the
# static power of those units when in use), and the HBM side
# one factor per execution unit (round 4): every group is driven by at least
# one single-unit calibration kernel of the power suite (csrc/apps/
# power_suite.hip), as AccelWattch calibrates each component on its own
# stress micro-benchmark; the unit mixes are held out for validation
UNIT_GROUPS: Dict[str, List[str]] = {
    "idle": ["CONSTP", "IDLE_COREP"],
    "static": ["STATICP"],
    # the core static power of SMs that issue (vs. that merely hold waves):
    # a latency-bound kernel keeps every CU resident and draws far less than
    # a compute-bound one (power_suite l2_read 485 W vs fp32_fma 1313 W)
    "static_issue": ["STATIC_ISSUEP"],
    "frontend": ["IBP", "ICP", "SCHEDP", "PIPEP", "RFP", "CCP"],
    "int": ["INTP", "INT_MULP", "INT_MUL24P", "INT_MUL32P", "INT_DIVP"],
    "fp": ["FPUP", "FP_DIVP", "FP_MULP", "FP_SQRTP", "FP_LGP", "FP_SINP", "FP_EXP"],
    "fp64": ["DPUP", "DP_MULP", "DP_DIVP"],
    "tensor": ["TENSORP", "TEXP"],
    # the memory units: LDS, L1, L2 accesses, their "in use" static power and
    # the fabric / HBM traffic (separate factors are not identifiable from the
    # single-unit kernels: each memory kernel drives several of them)
    "memory": ["SHRDP", "DCP", "TCP", "L2CP", "NOCP", "STATIC_MEMP", "DRAMP", "MCP"],
}

POWER_GROUPS: Dict[str, List[str]] = {
    "idle_static": ["CONSTP", "IDLE_COREP", "STATICP"],
    "valu": FINE_GROUPS["frontend"] + FINE_GROUPS["valu"] + FINE_GROUPS["sfu"] + FINE_GROUPS["fp64"],
    "tensor": FINE_GROUPS["tensor"],
    "memory": FINE_GROUPS["lds"] + FINE_GROUPS["cache"] + ["STATIC_MEMP"],
    "dram": FINE_GROUPS["dram"],
}


def fit_groups_relative(A: np.ndarray, b: np.ndarray, groups: Dict[str, List[str]] = FINE_GROUPS,
                        **kw) -> np.ndarray:
    """Group factors minimising the RELATIVE error (MAPE is the reported
    metric): rows scaled by 1 / measured power, target all ones."""
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    return fit_groups(A / b[:, None], np.ones(len(b)), groups=groups, **kw)


def governor_ratio(a_row: np.ndarray, x: np.ndarray, cap: float, v_floor: float, s_min: float = 0.5) -> float:
    """The DVFS governor of csrc/power/power.cc (dvfs_clock_ratio) on one
    kernel: the highest clock ratio in [s_min, 1] whose power fits the cap."""
    p = lambda s: float(a_row @ (x * dvfs_scale(s, v_floor, n=len(x))))
    if cap <= 0 or p(1.0) <= cap:
        return 1.0
    lo, hi = s_min, 1.0
    if p(lo) >= cap:
        return lo
    for _ in range(40):
        m = 0.5 * (lo + hi)
        if p(m) <= cap:
            lo = m
        else:
            hi = m
    return lo


def leave_one_out_dvfs(A: np.ndarray, b: np.ndarray, ratios: Sequence[float], v_floor: float, cap: float,
                       s_min: float = 0.5, **kw) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Leave-one-out over the kernels with the DVFS model.  Each fold fits the
    group factors on the other kernels at their MEASURED clocks, then
    predicts the held-out kernel (a) at its measured clock and (b) at the
    clock the governor picks under the measured cap.  Returns (power at the
    measured clock, power under the governor, governor clock ratios)."""
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    r = np.asarray(ratios, np.float64)
    n = len(b)
    at_meas, at_gov, s_gov = np.zeros(n), np.zeros(n), np.zeros(n)
    Ad = dvfs_matrix(A, r, v_floor)
    for i in range(n):
        keep = np.arange(n) != i
        x = fit_groups_relative(Ad[keep], b[keep], **kw)
        at_meas[i] = Ad[i] @ x
        s_gov[i] = governor_ratio(A[i], x, cap, v_floor, s_min)
        at_gov[i] = A[i] @ (x * dvfs_scale(s_gov[i], v_floor, n=A.shape[1]))
    return at_meas, at_gov, s_gov


def v_floor_from_measurements(sclk_mhz: Sequence[float], mv: Sequence[float], max_sclk: float) -> Optional[float]:
    """V(s)/V(1) = v_floor + (1 - v_floor) s from measured (clock, rail
    voltage) pairs: a line fitted through them, evaluated at s = 0.  None
    when fewer than 3 distinct clocks carry a voltage reading."""
    f = np.asarray(sclk_mhz, np.float64)
    v = np.asarray(mv, np.float64)
    ok = np.isfinite(f) & np.isfinite(v) & (v > 0)
    if ok.sum() < 3 or np.ptp(f[ok]) < 50.0:
        return None
    slope, icpt = np.polyfit(f[ok], v[ok], 1)
    v1 = icpt + slope * max_sclk
    if v1 <= 0:
        return None
    return float(min(0.95, max(0.0, icpt / v1)))
