"""Vector-L1 data path throughput (-sim_l1_port_bytes / -sim_l1_addr_lanes_per_cycle)
and its micro-benchmark fit in the tuner (ub_bw_widths)."""
import os

import pytest

from accel_sim_framework_distributed_amd.tuner import tuner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNED = os.path.join(ROOT, "configs", "tuned", "AMD_Instinct_MI355X")


def test_measured_l1_bandwidth_parsed():
    m = tuner.measured_l1_bandwidth([os.path.join(ROOT, "profiles", "ubench_mi355x")])
    assert m == {4: 20.7, 8: 27.6, 16: 28.7}


@pytest.mark.slow
def test_data_path_limits_wide_loads():
    off = tuner.simulated_l1_bandwidth(TUNED, 0, widths=(16,))
    on = tuner.simulated_l1_bandwidth(TUNED, 48, widths=(16,))
    # 128-bit loads: 8 lines of 128 B per wave, 3 data-path cycles each
    assert on[16] < 0.7 * off[16]
    assert on[16] <= 128 / 3 + 1e-9
    # a narrower path never raises the bandwidth
    narrow = tuner.simulated_l1_bandwidth(TUNED, 32, widths=(16,))
    assert narrow[16] <= on[16]


def test_address_stage_costs_cycles(native, tmp_path):
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "bfs"), rodinia.bfs(2048, levels=2))
    base = sim.simulate(kl, "QV100", engine="cpu")
    port = sim.simulate(kl, "QV100", engine="cpu", extra={"-sim_l1_port_bytes": "32"})
    both = sim.simulate(kl, "QV100", engine="cpu", extra={"-sim_l1_port_bytes": "32",
                                                          "-sim_l1_addr_lanes_per_cycle": "4"})
    assert base.tot_insn == port.tot_insn == both.tot_insn
    assert base.tot_cycle <= port.tot_cycle <= both.tot_cycle
    assert both.tot_cycle > base.tot_cycle
