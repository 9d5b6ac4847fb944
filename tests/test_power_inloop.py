"""Power sampled inside the engine's cycle loop (-power_in_loop, engine.h
PwrArm, power_eval.h): the same samples, bit for bit, as the host-driven
slices (one engine run per sample), with per-issue charging of each unit
kind's active lanes (reference incexecstat, shader.cc:3226-3290; mcpat_cycle
in the cycle loop, power_interface.cc:52-188).  GPU twin:
tests/test_gpu_engine.py::test_power_in_kernel_gpu_equals_cpu."""
import re

import pytest


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    from accel_sim_framework_distributed_amd.power import xmlcfg
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tmp_path_factory.mktemp("pil")
    kl = rodinia.write_app(str(d / "hs"), rodinia.hotspot(256, 2, 2))
    xml = str(d / "aw.xml")
    xmlcfg.write_xml(xml, xmlcfg.default_params("QV100"))
    return d, kl, xml


def _run(env, extra):
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.models import presets
    d, kl, xml = env
    tag = "_".join(f"{k}{v}" for k, v in sorted(extra.items())).replace("-", "")
    rep = str(d / f"p_{tag}.log")
    args = presets.args_for("QV100", dict({"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml,
                                           "-gpgpu_runtime_stat": "200:0", "-power_report_file": rep}, **extra))
    s = _native.load().Simulator(args + ["-trace", kl], False)
    assert s.run() == 0
    return s, open(rep).read()


@pytest.mark.parametrize("threads", ["1", "3"])
def test_in_loop_equals_sliced(env, threads):
    a, ra = _run(env, {"-power_in_loop": "0", "-sim_cpu_threads": threads})
    b, rb = _run(env, {"-power_in_loop": "1", "-sim_cpu_threads": threads})
    assert ra == rb and "kernel_avg_power" in ra
    assert a.tot_cycle == b.tot_cycle
    n = int(re.search(r"^power_in_loop_samples: (\d+)", b.output, re.M).group(1))
    assert n >= 5
    assert "power_in_loop_samples" not in a.output


def test_per_issue_unit_charging(env):
    """each unit kind's lanes are charged at issue: hotspot's FFMA / FMUL go
    to the FP multiplier, its integer address arithmetic to the INT units"""
    _, r = _run(env, {})
    tot = {k: float(v) for k, v in re.findall(r"^gpu_tot_(\w+) = ([0-9.e+-]+)", r, re.M)}
    assert tot["FP_MUL_ACC"] > 0 and tot["INT_ACC"] > 0
    assert tot["FP_MUL_ACC"] + tot["FP_ACC"] + tot["INT_ACC"] + tot["INT_MUL_ACC"] <= tot["TOT_INST"] * 32 + 1
