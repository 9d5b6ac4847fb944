"""AccelWattch XML files: the subset of the schema the power model reads.

The reference's configs/tested-cfgs/*/accelwattch_*.xml carry ~600 lines of
McPAT inputs; our model (csrc/power/power.h) consumes only the per-activity
scaling factors, constant / idle-SM power and the categorical static powers,
so the files written here contain just those ``<param>`` entries inside the
same ``<component id="root">`` wrapper.  Reference XMLs load unchanged.
"""
from __future__ import annotations

import re
from typing import Dict

ACTIVITIES = ["TOT_INST", "FP_INT", "IC_H", "IC_M", "DC_RH", "DC_RM", "DC_WH", "DC_WM", "CC_H", "CC_M",
              "SHRD_ACC", "REG_RD", "REG_WR", "INT_ACC", "FP_ACC", "DP_ACC", "INT_MUL_ACC", "FP_MUL_ACC",
              "FP_SQRT_ACC", "FP_LG_ACC", "FP_SIN_ACC", "FP_EXP_ACC", "DP_MUL_ACC", "TENSOR_ACC", "TEX_ACC",
              "MEM_RD", "MEM_WR", "MEM_PRE", "L2_RH", "L2_RM", "L2_WH", "L2_WM", "NOC_A", "PIPE_A"]

STATIC = ["constant_power", "idle_core_power"] + \
    [f"static_{c}_{k}" for c in ("cat1", "cat2", "cat3", "cat4", "cat5", "cat6", "light") for k in ("flane", "addlane")] + \
    ["static_shared_flane", "static_l1_flane", "static_l2_flane"]

_PARAM = re.compile(r'<param\s+name\s*=\s*"([^"]+)"\s+value\s*=\s*"([^"]*)"')


def read_xml(path: str) -> Dict[str, float]:
    out = {}
    for k, v in _PARAM.findall(open(path).read()):
        try:
            out[k] = float(v)
        except ValueError:
            pass
    return out


def write_xml(path: str, params: Dict[str, float], comment: str = "") -> str:
    lines = ['<?xml version="1.0" ?>', "<!-- AccelWattch power model parameters (accel_sim_framework_distributed_amd)"]
    if comment:
        lines.append("     " + comment)
    lines += ["-->", '<component id="root" name="root">', '\t<component id="system" name="system">']
    keys = [k for k in ACTIVITIES + STATIC if k in params] + sorted(k for k in params if k not in ACTIVITIES + STATIC)
    for k in keys:
        lines.append(f'\t\t<param name="{k}" value="{params[k]:.9g}" />')
    lines += ["\t</component>", "</component>", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))
    return path


def default_params(preset: str) -> Dict[str, float]:
    """Uncalibrated starting point per preset (all activity factors 1.0;
    constant / idle / static powers sized to the part's TDP class).  Use
    power.calibrate to fit them to measured power."""
    p = {a: 1.0 for a in ACTIVITIES}
    if preset.upper() == "MI355X":
        # 1400 W board, 256 CUs; ~300 W measured with the chip idle
        # (profiles/ubench_mi355x/ub_power.log): HBM3E stacks, fabric, MALL
        p.update(constant_power=230.0, idle_core_power=0.3)
        cats = dict(cat1=(120.0, 3.0), cat2=(150.0, 3.5), cat3=(170.0, 4.0), cat4=(155.0, 3.5), cat5=(130.0, 3.0),
                    cat6=(380.0, 0.0), light=(20.0, 0.05))
        p.update(static_shared_flane=90.0, static_l1_flane=100.0, static_l2_flane=60.0)
        # architectural energy model inputs (energy_model = 1, csrc/power/arch_energy.cc):
        # N3-class compute dies, HBM3E, MFMA 16x16x32 = 128 MACs per lane
        p.update(core_tech_node=3.0, dram_pj_per_bit=2.5, tensor_macs_per_lane=128.0)
        # CDNA transcendentals (v_sqrt / v_log / v_sin / v_exp) run on the VALU
        # at a quarter of the FMA rate: per lane they cost about an FMA, not
        # the 4x of a separate SFU the base table assumes (power suite, round 4:
        # held-out MAPE 15.3 -> 14.6 %, integer factor 0.37 -> 1.01)
        for a in ("FP_SQRT_ACC", "FP_LG_ACC", "FP_SIN_ACC", "FP_EXP_ACC"):
            p[a] = 0.25
    else:
        # 250 W class Volta/Turing/Ampere boards, 80-ish SMs
        p.update(constant_power=32.0, idle_core_power=0.28)
        cats = dict(cat1=(15.0, 0.6), cat2=(18.5, 0.65), cat3=(19.0, 0.7), cat4=(18.5, 0.6), cat5=(14.5, 0.5),
                    cat6=(49.0, 0.0), light=(2.0, 0.004))
        p.update(static_shared_flane=31.0, static_l1_flane=35.0, static_l2_flane=17.0)
        p.update(core_tech_node=12.0, dram_pj_per_bit=3.9)
    # 0: the fixed per-access energy table (power.cc); 1: energies derived
    # from the simulated machine's geometry (McPAT / CACTI role)
    p["energy_model"] = 0.0
    for c, (f, a) in cats.items():
        p[f"static_{c}_flane"] = f
        p[f"static_{c}_addlane"] = a
    return p
