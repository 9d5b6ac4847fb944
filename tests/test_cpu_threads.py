"""CPU engine thread team (-sim_cpu_threads, csrc/engine/thread_team.h): the
units of a PDES epoch run on persistent host threads with one spin barrier
per epoch; every thread evaluates the epoch decision itself.  Results are
bit-identical for any thread count (the reference is single-threaded; this is
the host-side analogue of the GPU engine's persistent kernel)."""
import pytest


def _strip(s):
    skip = ("rate", "slowdown", "time")
    return {a: v for a, v in s.items() if not any(x in a for x in skip)}


@pytest.fixture(scope="module")
def apps(tmp_path_factory):
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tmp_path_factory.mktemp("thr")
    return {"hotspot": rodinia.write_app(str(d / "hs"), rodinia.hotspot(64, 2, 2)),
            "bfs": rodinia.write_app(str(d / "bfs"), rodinia.bfs(2048, levels=3)),
            "backprop": rodinia.write_app(str(d / "bp"), rodinia.backprop(1024))}


@pytest.mark.parametrize("app", ["hotspot", "bfs", "backprop"])
@pytest.mark.parametrize("extra", [{}, {"-sim_xcd": "8", "-sim_mall": "256:16"}], ids=["shared_l2", "xcd_mall"])
def test_threads_bit_exact(apps, app, extra):
    from accel_sim_framework_distributed_amd import sim
    ref = sim.simulate(apps[app], "QV100", engine="cpu", extra=extra)
    for t in ("2", "3", "8"):
        r = sim.simulate(apps[app], "QV100", engine="cpu", extra=dict(extra, **{"-sim_cpu_threads": t}))
        assert (r.tot_cycle, r.tot_insn) == (ref.tot_cycle, ref.tot_insn), t
        assert _strip(r.stats) == _strip(ref.stats), t
        assert [k["cycles"] for k in r.kernels] == [k["cycles"] for k in ref.kernels]


def test_threads_state_image_and_power(apps, tmp_path):
    """full architectural state, the sampled power report and the DVFS
    governor's choices are identical with a team (power sampling stops and
    restarts the run at every sample)"""
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.power import report, xmlcfg
    xml = str(tmp_path / "aw.xml")
    xmlcfg.write_xml(xml, dict(xmlcfg.default_params("QV100"), power_cap=150.0, dvfs_v_floor=0.6))
    out = {}
    for thr in ("1", "4"):
        rep = str(tmp_path / f"p_{thr}.log")
        args = presets.args_for("QV100", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml,
                                          "-gpgpu_runtime_stat": "200:0", "-dvfs_enabled": "1",
                                          "-power_report_file": rep, "-sim_cpu_threads": thr}) + ["-trace", apps["hotspot"]]
        s = _native.load().Simulator(args, False)
        assert s.run() == 0
        out[thr] = (s.tot_cycle, report.parse_power_report(rep), s.snapshot(),
                    [l for l in s.output.splitlines() if l.startswith(("gpu_sim_time_ns", "gpu_avg_core_clock"))])
    assert out["1"] == out["4"]
    assert out["1"][1]


@pytest.mark.slow
def test_host_streamed_with_threads(tmp_path):
    """host-side trace streaming refills between epochs with the team parked
    at a barrier (thread 0 moves the window)"""
    import numpy as np
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("k_many", (3000, 1, 1), (256, 1, 1), nregs=16)
    base = k.g.gtid0.astype(np.int64) * 4
    k.op("LDG.E", [4], [2], base=0x7000_0000 + base, stride=4)
    k.alu("FFMA", 2, regs=(4, 5, 6))
    k.op("STG.E", [], [2, 4], base=0x9000_0000 + base, stride=4)
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "many"), [k.build()], text=True)
    a = sim.simulate(kl, "QV100", engine="cpu")
    b = sim.simulate(kl, "QV100", engine="cpu",
                     extra={"-trace_host_budget_mb": "0.2", "-gpu_trace_window": "1", "-sim_cpu_threads": "4"})
    assert (a.tot_cycle, a.tot_insn) == (b.tot_cycle, b.tot_insn)
    assert _strip(a.stats) == _strip(b.stats)
    assert "trace_host_streamed_kernels: 1" in b.output
