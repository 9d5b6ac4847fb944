"""Architectural energy model (McPAT / CACTI role, csrc/power/arch_energy.cc):
per-access energies from the machine's geometry and a technology node."""
import math

import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.power import report, xmlcfg
from test_power import _run


def _e(native, preset="QV100", extra=None, **kw):
    return native.arch_energy(presets.args_for(preset, extra or {}), **kw)


@pytest.mark.parametrize("preset,node", [("QV100", 12.0), ("MI355X", 3.0)])
def test_every_activity_priced(native, preset, node):
    d = _e(native, preset, node_nm=node)
    names = native.PowerModel.activity_names()
    assert list(d["base_nj"]) == names
    for k, v in d["base_nj"].items():
        assert math.isfinite(v) and v > 0, k
    for name, a in d["arrays"].items():
        assert a["read_nj"] > 0 and a["write_nj"] > 0 and a["area_mm2"] > 0 and a["leak_w"] > 0, name
        ndwl, ndbl, nspd, rows, cols = a["org"]
        assert ndwl >= 1 and ndbl >= 1 and rows >= 1 and cols >= 1
    # a DRAM column access costs more than any on-chip array access, a miss
    # more than the tag probe alone
    b = d["base_nj"]
    assert b["MEM_RD"] > max(b["DC_RH"], b["L2_RH"], b["REG_RD"], b["SHRD_ACC"])
    assert b["DC_RM"] > d["arrays"]["L1D"]["tag_nj"]
    assert "L2 slice" in d["report"] and "technology" in d["report"]


def test_geometry_moves_the_energies(native):
    base = _e(native)
    # a 4x larger L1 (more sets): dearer per access, more leakage and area
    big = _e(native, extra={"-gpgpu_cache:dl1": "S:16:128:64,L:L:m:N:L,A:512:8,16:0,32",
                            "-gpgpu_unified_l1d_size": "0", "-gpgpu_adaptive_cache_config": "0"})
    small = _e(native, extra={"-gpgpu_cache:dl1": "S:2:128:64,L:L:m:N:L,A:512:8,16:0,32",
                              "-gpgpu_unified_l1d_size": "0", "-gpgpu_adaptive_cache_config": "0"})
    for k in ("read_nj", "leak_w", "area_mm2"):
        assert big["arrays"]["L1D"][k] > small["arrays"]["L1D"][k], k
    assert big["base_nj"]["DC_RH"] > small["base_nj"]["DC_RH"]
    # the L1 does not touch the other units' energies
    assert big["base_nj"]["L2_RH"] == base["base_nj"]["L2_RH"]
    assert big["base_nj"]["REG_RD"] == base["base_nj"]["REG_RD"]


def test_technology_scaling(native):
    e12 = _e(native, node_nm=12.0)
    e7 = _e(native, node_nm=7.0)
    e45 = _e(native, node_nm=45.0)
    for k, v in e12["base_nj"].items():
        if k in ("MEM_RD", "MEM_WR", "MEM_PRE"):  # the DRAM device, not the core's node
            assert e7["base_nj"][k] == v
            continue
        assert e45["base_nj"][k] > v > e7["base_nj"][k], k
    # logic energy goes with Vdd^2 at a fixed node
    lo = _e(native, node_nm=12.0, vdd=0.6)
    hi = _e(native, node_nm=12.0, vdd=0.9)
    assert hi["base_nj"]["INT_ACC"] / lo["base_nj"]["INT_ACC"] == pytest.approx((0.9 / 0.6) ** 2, rel=1e-9)
    # DRAM energy per bit
    assert _e(native, dram_pj_per_bit=2.0)["base_nj"]["MEM_RD"] == pytest.approx(2.0 * 256e-3)


def test_scheduler_and_tensor_follow_the_machine(native):
    few = _e(native, extra={"-gpgpu_num_sched_per_core": "4"})
    many = _e(native, extra={"-gpgpu_num_sched_per_core": "1"})  # 4x the warps per scheduler
    assert many["base_nj"]["FP_INT"] > few["base_nj"]["FP_INT"]
    t32 = _e(native, tensor_macs_per_lane=32.0)["base_nj"]["TENSOR_ACC"]
    t128 = _e(native, tensor_macs_per_lane=128.0)["base_nj"]["TENSOR_ACC"]
    assert t128 > 3.5 * t32 * 0.9


def test_simulator_uses_the_model_when_the_xml_asks(native, tmp_path):
    p = xmlcfg.default_params("QV100")
    fixed_xml, arch_xml = str(tmp_path / "fixed.xml"), str(tmp_path / "arch.xml")
    xmlcfg.write_xml(fixed_xml, p)
    xmlcfg.write_xml(arch_xml, dict(p, energy_model=1, core_tech_node=12))
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    ks = [rodinia.vectoradd(300000)]
    s0, d0 = _run(native, tmp_path, "fixed", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": fixed_xml,
                                              "-gpgpu_perf_sim_memcpy": "0"}, ks)
    s1, d1 = _run(native, tmp_path, "arch", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": arch_xml,
                                             "-gpgpu_perf_sim_memcpy": "0"}, ks)
    assert (s0.tot_cycle, s0.tot_insn) == (s1.tot_cycle, s1.tot_insn)  # timing is untouched
    t1 = open(d1 / "accelwattch_power_report.log").read()
    assert "architectural energy model" in t1 and "L1D" in t1
    assert "architectural energy model" not in open(d0 / "accelwattch_power_report.log").read()
    r0 = report.parse_power_report(str(d0 / "accelwattch_power_report.log"))[0]
    r1 = report.parse_power_report(str(d1 / "accelwattch_power_report.log"))[0]
    # same static / constant terms, different per-access energies
    assert r0["avg"]["CONSTP"] == pytest.approx(r1["avg"]["CONSTP"])
    assert r0["avg"]["DRAMP"] != pytest.approx(r1["avg"]["DRAMP"])
    d = _e(native, node_nm=12.0)
    # DRAM power scales with the per-access energy ratio (same activity)
    ratio = d["base_nj"]["MEM_RD"] / native.PowerModel.base_nj(native.PowerModel.activity_names().index("MEM_RD"))
    assert r1["avg"]["DRAMP"] / r0["avg"]["DRAMP"] == pytest.approx(ratio, rel=0.15)
