"""Trace ingest on the MI355X matrix cores (csrc/engine/ingest_mfma.hip).

The device coalescer computes each shared-memory instruction's bank-conflict
degree and each global instruction's sorted line/sector list as one-hot
products on v_mfma_f32_32x32x16_bf16; instructions outside its windows go to
the host code.  The oracle is the host coalescer (trace.cc coalesce_kernel,
itself pinned to the reference semantics in test_trace_and_sim.py): the
instruction and access arrays must be byte-identical.
"""
import os
import random

import pytest


def test_host_only_build_reports_not_run(native, qv100_args):
    # without a visible device the entry point declines (callers keep the host path)
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible: covered by the gpu tests below")
    except ImportError:
        pass
    r = native.ingest_compare_lanes([("shared", 4, 0xF, [0, 4, 8, 12], "")], qv100_args, 0)
    assert r["ran"] is False


@pytest.fixture(scope="module")
def gpu_native():
    import torch  # bind torch's HIP runtime first
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    from accel_sim_framework_distributed_amd import _native
    mod = _native.load(prefer_torch_runtime=True)
    assert mod.gpu_available(), "HIP device not usable (native code must run, no silent fallback)"
    return mod


def _lanes(mask):
    return [i for i in range(64) if mask >> i & 1]


LDS_OPS = {4: ["ds_read_b32", "ds_write_b32", "ds_read2_b32", "ds_add_u32"], 8: ["ds_read_b64", "ds_write_b64",
            "ds_read2_b64", "ds_read_b64_tr_b16"], 12: ["ds_read_b96", "ds_write_b96"], 16: ["ds_read_b128",
            "ds_write_b128"], 1: ["ds_read_u8"], 2: ["ds_read_u16"]}


def _patterns(ws, rng):
    full = (1 << ws) - 1
    out = []

    def sh(width, mask, addrs):
        # wave64 traces carry CDNA opcodes (lane-group banking), wave32 SASS-style ones
        op = rng.choice(LDS_OPS[width]) if ws == 64 else ""
        out.append(("shared", width, mask, addrs, op))

    # shared memory: strides (conflict degree 1..ws), broadcast, multi-word, partial masks, random in 16 KB
    for stride in (1, 2, 3, 4, 8, 16, 17, 32, 33, 64):
        for width in (4, 8, 16):
            sh(width, full, [l * stride * 4 for l in range(ws)])
    sh(4, full, [128] * ws)
    sh(4, full, [(l % 4) * 4 for l in range(ws)])
    sh(4, full, [(l // 2) * 128 for l in range(ws)])
    sh(12, full, [l * 12 + 2 for l in range(ws)])
    for _ in range(60):
        m = rng.getrandbits(ws) or 1
        w = rng.choice((1, 2, 4, 8, 12, 16))
        sh(w, m, [rng.randrange(0, 16384) for _ in _lanes(m)])
    sh(4, full, [rng.randrange(0, 1 << 20) * 4 for _ in range(ws)])  # wide rows: host fallback
    # global: coalesced, strided, unaligned line-crossing, random inside / outside the 64-line window
    base = 0x7F1234560000
    for stride in (4, 8, 16, 32, 64, 128, 132, 256):
        for width in (1, 4, 8, 16):
            out.append(("global", width, full, [base + l * stride for l in range(ws)], ""))
    out.append(("global", 16, full, [base + 120 + l * 16 for l in range(ws)], ""))
    out.append(("global", 4, full, [base] * ws, ""))
    for _ in range(40):
        m = rng.getrandbits(ws) or 1
        w = rng.choice((1, 2, 4, 8, 16))
        span = rng.choice((512, 4096, 8000, 1 << 20))
        out.append(("global", w, m, [base + rng.randrange(0, span) for _ in _lanes(m)], ""))
    return out


def test_cdna_lane_group_banking(native):
    """MI355X LDS table: conflicts count per lane group of each ds_* form."""
    from accel_sim_framework_distributed_amd.models import presets
    args = presets.args_for("MI355X")
    full = (1 << 64) - 1
    deg = lambda addrs, w, op, m=full: native.smem_conflict_degree_cdna(addrs, m, w, op, args)  # noqa: E731
    lin4 = [4 * l for l in range(64)]
    assert deg(lin4, 4, "ds_read_b32") == 1
    # stride 2 dwords: each 32-lane half puts two words on every even bank of 32 -> 2-way in both halves
    assert deg([8 * l for l in range(64)], 4, "ds_read_b32") == 1 + 2
    # lanes l and l+32 on one bank never conflict; l and l+16 do (b32: 32 banks)
    assert deg([4 * (l % 32) + 128 * (l // 32) * 2 for l in range(64)], 4, "ds_read_b32") == 1
    assert deg([4 * (l % 16) + 64 * 4 * (l // 16) for l in range(64)], 4, "ds_read_b32") == 1 + 2
    # 8-byte reads use 64 banks, 8-byte stores 16-lane groups over 32 banks: both conflict-free when linear
    assert deg([8 * l for l in range(64)], 8, "ds_read_b64") == 1
    assert deg([8 * l for l in range(64)], 8, "ds_write_b64") == 1
    # b128 linear is conflict-free in its four interleaved 16-lane groups; rows of 256 B (bf16 D=128
    # row-major, lane = row) put the 16 lanes of a group on the same four banks: 16-way
    assert deg([16 * l for l in range(64)], 16, "ds_read_b128") == 1
    assert deg([256 * l for l in range(64)], 16, "ds_read_b128") == 1 + 4 * 15
    # broadcast
    assert deg([0] * 64, 4, "ds_read_b32") == 1
    # the GPGPU-Sim model (no lane groups) on the same stride-2 access: one 64-bank part, 2-way
    assert native.smem_conflict_degree([8 * l for l in range(64)], full, 4, args) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["QV100", "MI355X"])
def test_ingest_lanes_device_equals_host(gpu_native, preset):
    from accel_sim_framework_distributed_amd.models import presets
    args = presets.args_for(preset)
    ws = 64 if preset == "MI355X" else 32
    rng = random.Random(7 + ws)
    ins = _patterns(ws, rng)
    r = gpu_native.ingest_compare_lanes(ins, args, 0)
    assert r["ran"], r
    assert r["equal"], r
    # the matrix cores carried the regular patterns, the host only the out-of-window ones
    assert r["smem_device"] > 0.8 * (r["smem_device"] + r["smem_host"]), r
    assert r["gmem_device"] > 0.7 * (r["gmem_device"] + r["gmem_host"]), r
    assert r["smem_host"] >= 1 and r["gmem_host"] >= 1, r
    assert r["mfma"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["QV100", "MI355X"])
def test_ingest_suite_device_equals_host(gpu_native, preset, tmp_path):
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    args = presets.args_for(preset)
    kl = rodinia.generate_suite(str(tmp_path / "suite"))
    checked = 0
    dev = 0
    for app, path in sorted(kl.items()):
        d = os.path.dirname(path)
        for fn in sorted(os.listdir(d)):
            if not (fn.endswith(".asimk") or fn.endswith(".traceg")):
                continue
            r = gpu_native.ingest_compare(os.path.join(d, fn), args, 0)
            assert r["ran"], (app, fn)
            assert r["equal"], (app, fn, r)
            checked += 1
            dev += r["smem_device"] + r["gmem_device"]
    assert checked >= 11 and dev > 0


@pytest.mark.gpu
def test_simulation_with_device_ingest_equals_cpu(gpu_native, tmp_path):
    # -gpu_ingest 1 (the GPU engine's default) vs the CPU engine's host ingest
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "lud"), rodinia.lud(n=64))
    g = sim.simulate(kl, "QV100", engine="gpu", extra={"-gpu_ingest": "1", "-gpu_ingest_min_insts": "0"})
    c = sim.simulate(kl, "QV100", engine="cpu")
    assert (g.tot_insn, g.tot_cycle) == (c.tot_insn, c.tot_cycle)
    assert "gpu_ingest: shared" in g.output


def _lds_conflict_kernel():
    """wave64: ds_read_b128 on 256 B rows (16-way in each of its four lane
    groups: 60 extra cycles), ds_read_b32 at an 8 B stride (2-way in both
    32-lane halves: 2), ds_write_b64 at 8 B (conflict-free in 16-lane groups)."""
    import numpy as np
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("k_lds", (64, 1, 1), (256, 1, 1), nregs=32, binary_version=950, warp_size=64, shmem=65536)
    w = k.g.warp.astype(np.int64) % 4 * 16384
    k.op("ds_read_b128", [4], [2], base=w, stride=256)
    k.op("ds_read_b32", [5], [2], base=w, stride=8)
    k.op("ds_write_b64", [], [4], base=w, stride=8)
    k.op("s_waitcnt", [], [])
    k.op("s_endpgm")
    return k.build()


def _bkconflict(out):
    import re
    return int(re.findall(r"gpgpu_n_shmem_bkconflict = (\d+)", out)[-1])


def test_cdna_lane_groups_in_simulation(tmp_path):
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "lds"), [_lds_conflict_kernel()], memcpy=False)
    c = sim.simulate(kl, "MI355X", engine="cpu")
    assert _bkconflict(c.output) == 256 * (60 + 2)
    off = sim.simulate(kl, "MI355X", engine="cpu", extra={"-gpgpu_shmem_cdna_lane_groups": "0"})
    assert _bkconflict(off.output) != _bkconflict(c.output)


@pytest.mark.gpu
def test_cdna_lane_groups_gpu_equals_cpu(gpu_native, tmp_path):
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "lds"), [_lds_conflict_kernel()], memcpy=False)
    g = sim.simulate(kl, "MI355X", engine="gpu", extra={"-gpu_ingest_min_insts": "0"})
    c = sim.simulate(kl, "MI355X", engine="cpu")
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    assert _bkconflict(g.output) == _bkconflict(c.output) == 256 * (60 + 2)
    assert "gpu_ingest: shared" in g.output
