"""Issue stage: dual issue (-gpgpu_max_insn_issue_per_warp 2 with
-gpgpu_dual_issue_diff_exec_units, reference scheduler_unit::cycle
shader.cc:1249-1556), the warp-limiting and two-level schedulers
(shader.cc:1599-1700)."""
import re

import numpy as np
import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen import rodinia
from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder


def _run(native, kl, extra, preset="QV100"):
    s = native.Simulator(presets.args_for(preset, extra) + ["-trace", kl, "-gpgpu_perf_sim_memcpy", "0"], False)
    assert s.run() == 0
    return s


def _stat(out, key):
    m = re.findall(rf"{re.escape(key)} = ([0-9.]+)", out)
    return int(float(m[-1])) if m else 0


@pytest.fixture(scope="module")
def alu_pairs(tmp_path_factory):
    # one warp: 64 independent (FFMA, IMAD) pairs -- SP and INT units
    k = KernelBuilder("_Z4pairv", (1, 1, 1), (32, 1, 1), nregs=64)
    for i in range(64):
        k.op("FFMA", [8 + i % 8], [4, 5, 6])
        k.op("IMAD", [20 + i % 8], [4, 5, 6])
    k.op("EXIT")
    return rodinia.write_app(str(tmp_path_factory.mktemp("dual") / "pairs"), [k.build()], memcpy=False)


WIDE = {"-gpgpu_operand_collector_num_units_gen": "16", "-gpgpu_sub_core_model": "0",
        "-gpgpu_reg_file_port_throughput": "4", "-gpgpu_kernel_launch_latency": "0",
        "-trace_opcode_latency_initiation_sp": "2,1", "-trace_opcode_latency_initiation_int": "2,1"}


def test_dual_issue_pairs_different_units(native, alu_pairs):
    # a back end wide enough that the issue stage is the bottleneck
    one = _run(native, alu_pairs, dict(WIDE, **{"-gpgpu_max_insn_issue_per_warp": "1"}))
    two = _run(native, alu_pairs, dict(WIDE, **{"-gpgpu_max_insn_issue_per_warp": "2"}))
    assert _stat(one.output, "gpgpu_n_dual_issue") == 0
    assert _stat(two.output, "gpgpu_n_dual_issue") > 0
    assert two.tot_insn == one.tot_insn
    assert two.tot_cycle < one.tot_cycle


def test_dual_issue_same_unit_never_pairs(native, tmp_path):
    k = KernelBuilder("_Z4samev", (1, 1, 1), (32, 1, 1), nregs=64)
    for i in range(64):
        k.op("FFMA", [8 + i % 8], [4, 5, 6])
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "same"), [k.build()], memcpy=False)
    two = _run(native, kl, {"-gpgpu_max_insn_issue_per_warp": "2", "-gpgpu_dual_issue_diff_exec_units": "1"})
    assert _stat(two.output, "gpgpu_n_dual_issue") == 0


@pytest.fixture(scope="module")
def many_warps(tmp_path_factory):
    # 2 CTAs x 16 warps of loads and dependent math (warps stall on memory)
    k = KernelBuilder("_Z4manyPi", (2, 1, 1), (512, 1, 1), nregs=32)
    base = 0x7100_0000 + np.arange(k.g.nwarps, dtype=np.int64) * 4096
    for i in range(8):
        k.op("LDG.E", [8], [4], base=base + 128 * i, stride=4)
        k.op("FFMA", [9], [8, 5, 6])
        k.op("FFMA", [10], [9, 5, 6])
    k.op("EXIT")
    return rodinia.write_app(str(tmp_path_factory.mktemp("sched") / "many"), [k.build()], memcpy=False)


@pytest.mark.parametrize("sched", ["warp_limiting:2:1", "warp_limiting:2:2", "two_level_active:2:0:1",
                                   "two_level_active:6:0:1"])
def test_limited_schedulers_complete_and_differ(native, many_warps, sched):
    gto = _run(native, many_warps, {"-gpgpu_scheduler": "gto"})
    lim = _run(native, many_warps, {"-gpgpu_scheduler": sched})
    assert not lim.deadlock
    assert lim.tot_insn == gto.tot_insn
    if sched == "warp_limiting:2:1":
        # one warp at a time cannot hide the load latency
        assert lim.tot_cycle > gto.tot_cycle


def test_scheduler_parameters_are_checked(native):
    with pytest.raises(Exception):
        native.parse_config(presets.args_for("QV100", {"-gpgpu_scheduler": "warp_limiting:2"}))
    c = native.parse_config(presets.args_for("QV100", {"-gpgpu_scheduler": "two_level_active:6:0:1"}))
    assert c["sched_param"] == 6
