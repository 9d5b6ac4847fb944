"""Model switches of the reference that isolate parts of the memory system
(-gpgpu_perfect_mem, -gpgpu_simple_dram_model, DRAM scheduler choice) and the
run caps (-gpgpu_max_cycle / -gpgpu_max_insn)."""
import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen import rodinia


@pytest.fixture(scope="module")
def traces(tmp_path_factory):
    d = tmp_path_factory.mktemp("opts")
    return {"vadd": rodinia.write_app(str(d / "vadd"), [rodinia.vectoradd(200000)]),
            "bfs": rodinia.write_app(str(d / "bfs"), rodinia.bfs(2048))}


def _run(native, kl, extra):
    s = native.Simulator(presets.args_for("QV100", extra) + ["-trace", kl], False)
    assert s.run() == 0
    return s


def test_perfect_memory_is_faster_and_silent(native, traces):
    base = _run(native, traces["vadd"], {})
    pm = _run(native, traces["vadd"], {"-gpgpu_perfect_mem": "1"})
    assert pm.tot_insn == base.tot_insn
    assert pm.tot_cycle < base.tot_cycle
    assert "total dram reads = 0" in pm.output


def test_simple_dram_model_runs(native, traces):
    base = _run(native, traces["bfs"], {})
    sd = _run(native, traces["bfs"], {"-gpgpu_simple_dram_model": "1"})
    assert sd.tot_insn == base.tot_insn and sd.tot_cycle > 0


def test_dram_scheduler_choice_matters(native, traces):
    # cold L2 (no memcpy pre-fill): three streams in different DRAM rows interleave in the queues
    fr = _run(native, traces["vadd"], {"-gpgpu_dram_scheduler": "1", "-gpgpu_perf_sim_memcpy": "0"})
    ff = _run(native, traces["vadd"], {"-gpgpu_dram_scheduler": "0", "-gpgpu_perf_sim_memcpy": "0"})
    assert fr.tot_insn == ff.tot_insn
    assert fr.tot_cycle != ff.tot_cycle


def test_max_cycle_cap_breaks(native, traces):
    s = native.Simulator(presets.args_for("QV100", {"-gpgpu_max_cycle": "3000"}) + ["-trace", traces["bfs"]], False)
    assert s.run() == 0
    assert "break due to reaching the maximum cycles" in s.output
    full = _run(native, traces["bfs"], {})
    assert s.tot_insn < full.tot_insn
