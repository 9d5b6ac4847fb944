"""AccelWattch-compatible power model: sampling, report, HW/HYBRID modes, calibration."""
import os

import numpy as np
import pytest

from accel_sim_framework_distributed_amd.power import calibrate, report, xmlcfg
from conftest import reference_path


def _run(native, tmp_path, name, extra, kernels=None):
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tmp_path / name
    d.mkdir()
    kl = rodinia.write_app(str(d / "traces"), kernels or [rodinia.vectoradd(20000)])
    presets.write_config("QV100", str(tmp_path / "cfg"))
    args = presets.args_for("QV100", extra) + ["-trace", kl]
    cwd = os.getcwd()
    os.chdir(d)
    try:
        s = native.Simulator(args, False)
        assert s.run() == 0
    finally:
        os.chdir(cwd)
    return s, d


def test_power_sampling_does_not_change_timing(native, tmp_path):
    xml = str(tmp_path / "aw.xml")
    xmlcfg.write_xml(xml, xmlcfg.default_params("QV100"))
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    ks = [rodinia.vectoradd(300000)]
    base, _ = _run(native, tmp_path, "plain", {}, ks)
    pw, d = _run(native, tmp_path, "power", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml,
                                             "-gpgpu_runtime_stat": "300:0", "-power_trace_enabled": "1",
                                             "-steady_power_levels_enabled": "1"}, ks)
    assert pw.tot_cycle == base.tot_cycle and pw.tot_insn == base.tot_insn
    ks = report.parse_power_report(str(d / "accelwattch_power_report.log"))
    assert len(ks) == 1
    k = ks[0]
    assert k["kernel_avg_power"] > xmlcfg.default_params("QV100")["constant_power"]
    assert abs(sum(k["avg"].values()) - k["kernel_avg_power"]) < 1e-4 * k["kernel_avg_power"]
    assert k["kernel_max_power"] >= k["kernel_avg_power"] >= k["kernel_min_power"]
    assert k["avg"]["DRAMP"] > 0 and k["avg"]["IBP"] > 0
    trace = open(d / "accelwattch_power_trace.csv").read().splitlines()
    assert trace[0].startswith("cycle,total_power") and len(trace) > 3   # several samples
    assert "gpu_avg_power" in pw.output


def test_power_hw_and_hybrid_modes(native, tmp_path):
    xml = str(tmp_path / "aw.xml")
    xmlcfg.write_xml(xml, xmlcfg.default_params("QV100"))
    sim, d0 = _run(native, tmp_path, "sim", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml})
    kname = sim.kernels[0]["name"]
    csv = tmp_path / "hw_perf.csv"
    csv.write_text("Benchmark,Kernel,L1_RH,L1_RM,L1_WH,L1_WM,CC_ACC,SHRD_ACC,DRAM_Rd,DRAM_Wr,L2_RH,L2_RM,L2_WH,L2_WM,"
                   "NOC,Pipeline_Duty,Num_Idle_SMs,Elapsed_Cycles,Chip Voltage\n"
                   f"vadd,{kname},100,100,0,0,0,0,9000000,9000000,0,0,0,0,1000,0.5,10,20000,1.0\n")
    common = {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml, "-hw_perf_file_name": str(csv),
              "-hw_perf_bench_name": "vadd"}
    hw, d1 = _run(native, tmp_path, "hw", dict(common, **{"-power_simulation_mode": "1"}))
    hy, d2 = _run(native, tmp_path, "hy", dict(common, **{"-power_simulation_mode": "2",
                                                           "-accelwattch_hybrid_perfsim_DRAM_RD": "1",
                                                           "-accelwattch_hybrid_perfsim_DRAM_WR": "1"}))
    r0 = report.parse_power_report(str(d0 / "accelwattch_power_report.log"))[0]
    r1 = report.parse_power_report(str(d1 / "accelwattch_power_report.log"))[0]
    r2 = report.parse_power_report(str(d2 / "accelwattch_power_report.log"))[0]
    # HW mode takes the (huge) DRAM counts from the csv; HYBRID keeps the simulated ones
    assert r1["avg"]["DRAMP"] > 10 * r0["avg"]["DRAMP"]
    assert r2["avg"]["DRAMP"] < r1["avg"]["DRAMP"] / 10
    # HW mode: a single sample per kernel
    assert r1["kernel_max_power"] == pytest.approx(r1["kernel_min_power"])


def test_reference_xml_loads(native, tmp_path):
    ref = reference_path("gpu-simulator", "gpgpu-sim", "configs", "tested-cfgs", "SM7_QV100", "accelwattch_sass_sim.xml")
    if ref is None:
        pytest.skip("reference configs not mounted")
    p = xmlcfg.read_xml(ref)
    assert p["TOT_INST"] == 10 and "static_cat6_flane" in p
    s, d = _run(native, tmp_path, "refxml", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": ref})
    assert report.parse_power_report(str(d / "accelwattch_power_report.log"))[0]["kernel_avg_power"] > 0


def test_calibration_recovers_factors():
    rng = np.random.default_rng(7)
    n_k, comps = 40, len(report.COMPONENTS)
    A = np.zeros((n_k, comps))
    active = rng.choice(comps, 14, replace=False)
    A[:, active] = rng.uniform(0.5, 30.0, (n_k, len(active)))
    x_true = np.ones(comps)
    x_true[active] = rng.uniform(0.3, 3.0, len(active))
    b = A @ x_true * (1 + rng.normal(0, 0.002, n_k))
    x = calibrate.fit_scaling(A, b, lower=0.05, upper=100)
    assert np.allclose(x[active], x_true[active], rtol=0.2)
    pred = calibrate.leave_one_out(A, b, lower=0.05, upper=100)
    err, _ = calibrate.mape(pred, b)
    assert err < 3.0
    # an ordering constraint x[a0] <= x[a1] is honoured
    a0, a1 = active[0], active[1]
    C = np.zeros((1, comps))
    C[0, a0], C[0, a1] = 1.0, -1.0
    xc = calibrate.fit_scaling(A, b, lower=0.05, upper=100, C=C, d=np.zeros(1))
    assert xc[a0] <= xc[a1] + 1e-6


def test_grouped_fit_shares_factors():
    rng = np.random.default_rng(3)
    A = rng.uniform(0, 10, (12, len(report.COMPONENTS)))
    x_true = calibrate.group_matrix()[1].T @ np.array([1.2, 0.8, 1.5, 0.6, 2.0])
    x_true[x_true == 0] = 1.0
    b = A @ x_true
    x = calibrate.fit_groups(A, b, lower=0.05, upper=50)
    assert np.allclose(A @ x, b, rtol=1e-6)


@pytest.mark.slow
def test_mi355x_power_validation_pipeline(native, tmp_path):
    """Synthetic CDNA traces of the ub_power kernels -> simulated component
    power -> grouped QP fit against the amd-smi measurements."""
    from accel_sim_framework_distributed_amd.power import mi355x_validation as v
    s = v.run(str(tmp_path / "w"), str(tmp_path / "cal.xml"), iters=6)
    assert set(s["kernels"]) == {"idle", "fp32_fma", "int32_mad", "fp64_fma", "sfu_sqrt_exp", "mfma_bf16",
                                 "lds_read", "hbm_read"}
    assert s["mape_in_sample"] <= s["mape_uncalibrated"] + 1e-9
    assert os.path.exists(tmp_path / "cal.xml") and xmlcfg.read_xml(str(tmp_path / "cal.xml"))["constant_power"] > 0


def test_apply_factors_rescales_xml(tmp_path):
    src = str(tmp_path / "in.xml")
    xmlcfg.write_xml(src, xmlcfg.default_params("MI355X"))
    x = np.ones(len(report.COMPONENTS))
    x[report.COMPONENTS.index("DRAMP")] = 2.0
    x[report.COMPONENTS.index("STATICP")] = 0.5
    out = str(tmp_path / "out.xml")
    calibrate.apply_factors(src, out, x)
    p0, p1 = xmlcfg.read_xml(src), xmlcfg.read_xml(out)
    assert p1["MEM_RD"] == pytest.approx(2 * p0["MEM_RD"]) and p1["MEM_WR"] == pytest.approx(2 * p0["MEM_WR"])
    assert p1["static_cat2_flane"] == pytest.approx(0.5 * p0["static_cat2_flane"])
    assert p1["INT_ACC"] == pytest.approx(p0["INT_ACC"])


@pytest.mark.slow
def test_capped_fit_recovers_power_cap():
    # synthetic suite: linear model with known group factors, clipped at a cap
    rng = np.random.RandomState(3)
    comps = list(calibrate.COMPONENTS)
    A = np.zeros((24, len(comps)))
    A[:, comps.index("CONSTP")] = 300.0
    A[:, comps.index("FPUP")] = rng.uniform(0, 400, 24)
    A[:, comps.index("DRAMP")] = rng.uniform(0, 150, 24)
    A[:, comps.index("TENSORP")] = rng.uniform(0, 100, 24) * (rng.rand(24) < 0.4)
    x_true = np.ones(len(comps))
    x_true[comps.index("FPUP")] = 2.5
    x_true[comps.index("DRAMP")] = 3.0
    x_true[comps.index("TENSORP")] = 6.0
    b = np.minimum(A @ x_true, 1200.0)
    assert (A @ x_true > 1200.0).sum() >= 3  # some kernels really are capped
    x, cap = calibrate.fit_groups_capped(A, b, restarts=3)
    assert cap == pytest.approx(1200.0, rel=5e-3)
    assert calibrate.mape(calibrate.predict_capped(A, x, cap), b)[0] < 0.5
    loo = calibrate.leave_one_out_capped(A, b, restarts=2)
    assert calibrate.mape(loo, b)[0] < 2.0


def _cap_setup(native, tmp_path):
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    p = xmlcfg.default_params("QV100")
    free_xml = str(tmp_path / "free.xml")
    xmlcfg.write_xml(free_xml, p)
    ks = rodinia.hotspot(512, 2, 1)
    opts = {"-power_simulation_enabled": "1", "-gpgpu_runtime_stat": "200:0", "-power_trace_enabled": "1"}
    free_sim, d0 = _run(native, tmp_path, "free", dict(opts, **{"-accelwattch_xml_file": free_xml}), ks)
    free = report.parse_power_report(str(d0 / "accelwattch_power_report.log"))[0]
    cap = 0.5 * (free["kernel_max_power"] + free["kernel_avg_power"])
    capped_xml = str(tmp_path / "capped.xml")
    xmlcfg.write_xml(capped_xml, dict(p, power_cap=cap, dvfs_v_floor=0.6))
    return ks, opts, free_sim, free, cap, capped_xml


def test_power_cap_without_dvfs_reports_the_estimate(native, tmp_path):
    """A power limit alone changes nothing: the report is the activity's power
    (no rescaling to the cap -- only the DVFS governor can hold the cap)."""
    ks, opts, free_sim, free, cap, capped_xml = _cap_setup(native, tmp_path)
    assert free["kernel_max_power"] > cap
    s, d1 = _run(native, tmp_path, "capped", dict(opts, **{"-accelwattch_xml_file": capped_xml}), ks)
    k = report.parse_power_report(str(d1 / "accelwattch_power_report.log"))[0]
    assert s.tot_cycle == free_sim.tot_cycle
    assert k["kernel_avg_power"] == pytest.approx(free["kernel_avg_power"], rel=1e-9)


def test_dvfs_governor_slows_the_clock_under_the_cap(native, tmp_path):
    """-dvfs_enabled with a measured power cap (reference gpgpu_sim_wrapper.cc:
    948-958 voltage scaling; here the clock drops too): samples over the cap
    make the governor lower the core clock and voltage, power falls towards
    the cap, and the kernel takes longer in simulated time."""
    ks, opts, free_sim, free, cap, capped_xml = _cap_setup(native, tmp_path)
    s, d1 = _run(native, tmp_path, "dvfs", dict(opts, **{"-accelwattch_xml_file": capped_xml,
                                                         "-dvfs_enabled": "1"}), ks)
    k = report.parse_power_report(str(d1 / "accelwattch_power_report.log"))[0]
    assert s.tot_insn == free_sim.tot_insn
    assert k["kernel_avg_clock_ratio"] < 0.99
    assert k["kernel_avg_power"] < free["kernel_avg_power"]
    assert k["kernel_max_power"] < free["kernel_max_power"]
    # steady state (the middle of the kernel): the governor holds the cap
    tr = [float(l.split(",")[1]) for l in open(d1 / "accelwattch_power_trace.csv").read().splitlines()[1:]]
    mid = tr[len(tr) // 3: 2 * len(tr) // 3]
    assert sum(mid) / len(mid) == pytest.approx(cap, rel=0.03)
    assert abs(sum(k["avg"].values()) - k["kernel_avg_power"]) < 1e-4 * k["kernel_avg_power"]
    import re
    mhz = float(re.search(r"gpu_avg_core_clock_mhz = ([0-9.]+)", s.output).group(1))
    t_ns = float(re.search(r"gpu_sim_time_ns = ([0-9.]+)", s.output).group(1))
    nominal = 1447.0  # QV100 core clock
    assert mhz < nominal * 0.999
    # simulated time: the free run's cycles at the nominal clock vs the DVFS run
    assert t_ns > free_sim.tot_cycle / nominal * 1e3
    # the memory clocks did not slow down: memory-bound phases take fewer
    # (slower) core cycles, so the cycle count differs from the free run
    assert s.tot_cycle != free_sim.tot_cycle


def test_dvfs_checkpoint_resume_reproduces_the_run(native, tmp_path):
    """The core-clock time base is part of the checkpoint: a resumed DVFS run
    matches the uninterrupted one cycle for cycle."""
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    p = xmlcfg.default_params("QV100")
    xml = str(tmp_path / "c.xml")
    kl = rodinia.write_app(str(tmp_path / "tr"), rodinia.pathfinder(4000, 12, 2))
    # a cap low enough that the governor is active in every kernel
    xmlcfg.write_xml(xml, dict(p, power_cap=p["constant_power"] * 1.02))
    base = presets.args_for("QV100", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml,
                                      "-dvfs_enabled": "1", "-gpgpu_runtime_stat": "200:0"}) + \
        ["-trace", kl, "-checkpoint_path", str(tmp_path / "ck"), "-power_report_file", str(tmp_path / "p.log")]
    full = native.Simulator(base, False)
    assert full.run() == 0
    c = native.Simulator(base + ["-checkpoint_option", "1", "-checkpoint_kernel", "2"], False)
    assert c.run() == 0
    r = native.Simulator(base + ["-resume_option", "1", "-resume_kernel", "2"], False)
    assert r.run() == 0
    fk = [(k["name"], k["cycles"], k["insn"]) for k in full.kernels]
    rk = [(k["name"], k["cycles"], k["insn"]) for k in r.kernels]
    assert fk[2:] == rk and r.tot_cycle == full.tot_cycle
    import re
    assert re.findall(r"gpu_sim_time_ns = ([0-9.]+)", full.output)[2:] == \
        re.findall(r"gpu_sim_time_ns = ([0-9.]+)", r.output)


def test_dvfs_calibration_recovers_factors_from_measured_clocks():
    """Synthetic suite throttled by a governor like the simulator's: with the
    measured clocks and cap the fit recovers the group factors, leave-one-out
    is accurate at the measured clock, and the governor predicts the clocks."""
    from accel_sim_framework_distributed_amd.power import mi355x_validation as v
    rng = np.random.RandomState(5)
    comps = list(calibrate.COMPONENTS)
    n = 28
    A = np.zeros((n, len(comps)))
    A[:, comps.index("CONSTP")] = 250.0
    A[:, comps.index("STATICP")] = rng.uniform(50, 150, n)
    A[:, comps.index("FPUP")] = rng.uniform(0, 500, n)
    A[:, comps.index("DRAMP")] = rng.uniform(0, 200, n)
    A[:, comps.index("TENSORP")] = rng.uniform(0, 300, n) * (rng.rand(n) < 0.4)
    x_true = np.ones(len(comps))
    x_true[comps.index("FPUP")] = 1.8
    x_true[comps.index("TENSORP")] = 2.5
    cap, vf = 1000.0, 0.55
    ratios = np.array([calibrate.governor_ratio(A[i], x_true, cap, vf, 0.4) for i in range(n)])
    assert (ratios < 0.98).sum() >= 4  # several kernels really throttle
    b = np.array([A[i] @ (x_true * calibrate.dvfs_scale(r, vf)) for i, r in enumerate(ratios)])
    fmax = 2400.0
    s = v.fit_report_dvfs(A, b, [f"k{i}" for i in range(n)], list(ratios * fmax), [float("nan")] * n, cap, fmax,
                          v_floor=vf)
    assert s["mape_in_sample"] < 0.5 and s["mape_leave_one_out"] < 1.0
    assert s["governor"]["mape_leave_one_out"] < 1.0 and s["governor"]["clock_ratio_mae"] < 0.01
    assert s["group_factors"]["valu"] == pytest.approx(1.8, rel=0.02)
    assert not s["factors_at_bound"]
    # the rail voltage line: V = 500 + 0.2 * f mV -> v_floor = 500 / (500 + 480)
    f = np.array([1500.0, 1800.0, 2100.0, 2400.0])
    assert calibrate.v_floor_from_measurements(f, 500 + 0.2 * f, 2400.0) == pytest.approx(500 / 980, rel=1e-6)
