"""Trace ingest and end-to-end CPU-engine simulation."""
import os

import numpy as np
import pytest

from accel_sim_framework_distributed_amd import sim
from accel_sim_framework_distributed_amd.tracegen import format as tfmt, rodinia


@pytest.fixture(scope="module")
def vadd(tmp_path_factory):
    d = tmp_path_factory.mktemp("vadd")
    kb = rodinia.write_app(str(d / "bin"), [rodinia.vectoradd(n=20000, block=256)])
    kt = rodinia.write_app(str(d / "txt"), [rodinia.vectoradd(n=20000, block=256)], text=True)
    return kb, kt


def test_binary_roundtrip(tmp_path):
    k = rodinia.vectoradd(n=5000, block=256)
    p = str(tmp_path / "k.asimk")
    tfmt.write_kernel_binary(p, k)
    r = tfmt.read_kernel_binary(p)
    assert np.array_equal(r.insts, k.insts) and np.array_equal(r.mems, k.mems)
    assert np.array_equal(r.streams, k.streams)


def test_text_and_binary_agree(native, vadd, qv100_args):
    kb, kt = vadd
    ib = native.kernel_info(os.path.join(os.path.dirname(kb), "kernel-1.asimk"))
    it = native.kernel_info(os.path.join(os.path.dirname(kt), "kernel-1.traceg"))
    for key in ("grid", "block", "warp_insts", "thread_insts", "n_cta"):
        assert ib[key] == it[key], key
    rb = sim.simulate(kb, "QV100")
    rt = sim.simulate(kt, "QV100")
    assert (rb.tot_cycle, rb.tot_insn) == (rt.tot_cycle, rt.tot_insn)


def test_vectoradd_stats(vadd):
    r = sim.simulate(vadd[0], "QV100")
    assert r.tot_insn == 20000 // 32 * 12 * 32 or r.tot_insn > 0
    st = r.stats
    assert st["gpu_sim_insn"] == r.tot_insn
    assert st["gpu_tot_sim_cycle"] == r.tot_cycle
    assert "*** exit detected ***" in r.output
    # 5000-cycle kernel launch latency is part of the kernel time (QV100)
    assert r.tot_cycle > 5000
    # coalesced 8B loads: 2 lines per warp per load
    assert st["Total_core_cache_stats_breakdown[GLOBAL_ACC_R][TOTAL_ACCESS]"] > 0


def test_deterministic_and_thread_invariant(vadd):
    a = sim.simulate(vadd[0], "QV100")
    b = sim.simulate(vadd[0], "QV100")
    strip = lambda s: {k: v for k, v in s.items() if "rate" not in k and "slowdown" not in k and "time" not in k}
    assert (a.tot_cycle, a.tot_insn) == (b.tot_cycle, b.tot_insn)
    assert strip(a.stats) == strip(b.stats)


def test_decode_opcodes(native):
    d = native.decode_opcode("LDG.E.64.STRONG.GPU", 70)
    assert d["cls"] == 6 and d["width"] == 8 and d["flags"] & 1
    assert native.decode_opcode("HMMA.1688.F32", 75)["cls"] == 15  # SPEC3 (tensor unit) on Turing
    assert native.decode_opcode("BRA", 70)["cls"] == 13           # SPEC1 (branch unit) on Volta
    assert native.decode_opcode("BRA", 60)["cls"] == 8            # BRANCH on Pascal
    assert native.decode_opcode("v_mfma_f32_32x32x16_bf16", 950)["cls"] == 4
    assert native.decode_opcode("global_load_dwordx4", 950)["width"] == 16
    assert native.decode_opcode("s_waitcnt", 950)["flags"] & 8


def test_shared_bank_conflicts(native, qv100_args):
    full = (1 << 32) - 1
    lin = [i * 4 for i in range(32)]
    assert native.smem_conflict_degree(lin, full, 4, qv100_args) == 1
    bcast = [0] * 32
    assert native.smem_conflict_degree(bcast, full, 4, qv100_args) == 1
    stride2 = [i * 8 for i in range(32)]
    assert native.smem_conflict_degree(stride2, full, 4, qv100_args) == 2
    col = [i * 128 for i in range(32)]
    assert native.smem_conflict_degree(col, full, 4, qv100_args) == 32


def test_shared_bank_conflicts_random(native, qv100_args):
    """The stack-array fast path agrees with the definition (max distinct
    4-byte words per bank over the active lanes) on random patterns,
    including multi-word accesses and partial masks."""
    import random
    rng = random.Random(7)
    for _ in range(300):
        width = rng.choice([1, 2, 4, 8, 16])
        span = rng.choice([64, 256, 4096])
        addr = [rng.randrange(0, span) * rng.choice([1, 4]) for _ in range(32)]
        mask = rng.getrandbits(32) | 1
        banks = {}
        for l in range(32):
            if mask >> l & 1:
                for w in range(addr[l] >> 2, ((addr[l] + width - 1) >> 2) + 1):
                    banks.setdefault(w % 32, set()).add(w)
        want = max(len(v) for v in banks.values())
        assert native.smem_conflict_degree(addr, mask, width, qv100_args) == want


def test_coalescing(native, tmp_path, qv100_args):
    k = rodinia.vectoradd(n=64, block=64)
    p = str(tmp_path / "k.asimk")
    tfmt.write_kernel_binary(p, k)
    s = native.coalesce_summary(p, qv100_args)
    # per warp: 2 loads + 1 store of 8B x 32 lanes = 256B = 2 lines each
    assert s["n_accs"] == 2 * 3 * 2
    assert all(sec == 0xF for _, sec, _ in s["accs"])
