"""Timing-state checkpoint / resume at kernel boundaries: a run
resumed from the checkpoint after kernel K reproduces the uninterrupted run's
remaining kernels cycle-for-cycle, on either engine."""
import os

import pytest


def _sims(native, tmp_path, engine_ckpt, engine_resume):
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "tr"), rodinia.pathfinder(4000, 12, 2))
    base = presets.args_for("QV100") + ["-trace", kl, "-checkpoint_path", str(tmp_path / "ck")]
    full = native.Simulator(base + ["-sim_engine", engine_resume], False)
    assert full.run() == 0
    c = native.Simulator(base + ["-sim_engine", engine_ckpt, "-checkpoint_option", "1", "-checkpoint_kernel", "2"],
                         False)
    assert c.run() == 0
    assert os.path.exists(tmp_path / "ck" / "asim_state_kernel2.ckpt")
    r = native.Simulator(base + ["-sim_engine", engine_resume, "-resume_option", "1", "-resume_kernel", "2"], False)
    assert r.run() == 0
    return full, c, r


def _check(full, r):
    fk = [(k["name"], k["cycles"], k["insn"]) for k in full.kernels]
    rk = [(k["name"], k["cycles"], k["insn"]) for k in r.kernels]
    assert len(rk) == len(fk) - 2
    assert fk[2:] == rk
    assert r.tot_cycle == full.tot_cycle and r.tot_insn == full.tot_insn


def test_checkpoint_resume_cpu(native, tmp_path):
    full, c, r = _sims(native, tmp_path, "cpu", "cpu")
    _check(full, r)
    assert "resumed from" in r.output


def test_checkpoint_rejects_other_config(native, tmp_path):
    from accel_sim_framework_distributed_amd.models import presets
    full, c, r = _sims(native, tmp_path, "cpu", "cpu")
    args = presets.args_for("RTX2060") + ["-trace", str(tmp_path / "tr" / "kernelslist.g"), "-checkpoint_path",
                                          str(tmp_path / "ck"), "-resume_option", "1", "-resume_kernel", "2"]
    s = native.Simulator(args, False)
    with pytest.raises(RuntimeError):
        s.run()


@pytest.mark.gpu
def test_checkpoint_gpu_to_cpu(native, tmp_path):
    if not native.gpu_available():
        pytest.fail("GPU engine not available on a GPU test run")
    # checkpoint written by the MI355X engine, resumed by the CPU engine
    full, c, r = _sims(native, tmp_path, "gpu", "cpu")
    _check(full, r)
