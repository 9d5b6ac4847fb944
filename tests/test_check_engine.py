"""Lock-step engine checker (`-sim_engine check`, csrc/engine/check_engine.cc)
on the CPU: the CPU engine checked against itself must agree at every check
point and give the plain run's result; a perturbed reference state must be
reported with its cycle.  (GPU vs CPU: tests/test_gpu_engine.py.)"""
import pytest

from accel_sim_framework_distributed_amd import sim
from accel_sim_framework_distributed_amd.tracegen import rodinia


@pytest.fixture(scope="module")
def nw(tmp_path_factory):
    d = tmp_path_factory.mktemp("nw")
    return rodinia.generate_suite(str(d), ["nw-rodinia-2.0-ft"])["nw-rodinia-2.0-ft"]


@pytest.mark.slow
def test_check_engine_self_consistent(native, nw):
    c = sim.simulate(nw, "QV100", engine="cpu")
    k = sim.simulate(nw, "QV100", engine="check", extra={"-sim_check_primary": "cpu", "-sim_check_interval": "300"})
    assert (k.tot_cycle, k.tot_insn) == (c.tot_cycle, c.tot_insn)


def test_check_engine_reports_divergence(native, nw):
    with pytest.raises(Exception, match="engine check failed at cycle"):
        sim.simulate(nw, "QV100", engine="check",
                     extra={"-sim_check_primary": "cpu", "-sim_check_interval": "300", "-sim_check_corrupt_at": "1000"})


def test_check_engine_reports_mailbox_divergence(native, nw):
    # a wrong mailbox count is caught at the check point where it happens and
    # named as a mailbox, not blamed on the unit that later receives it
    with pytest.raises(Exception, match="mailbox count diverges"):
        sim.simulate(nw, "QV100", engine="check",
                     extra={"-sim_check_primary": "cpu", "-sim_check_interval": "300", "-sim_check_corrupt_at": "1000",
                            "-sim_check_corrupt_mailbox": "1"})
