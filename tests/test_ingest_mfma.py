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
    r = native.ingest_compare_lanes([("shared", 4, 0xF, [0, 4, 8, 12])], qv100_args, 0)
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


def _patterns(ws, rng):
    full = (1 << ws) - 1
    out = []
    # shared memory: strides (conflict degree 1..ws), broadcast, multi-word, partial masks, random in 16 KB
    for stride in (1, 2, 3, 4, 8, 16, 17, 32, 33, 64):
        for width in (4, 8, 16):
            out.append(("shared", width, full, [l * stride * 4 for l in range(ws)]))
    out.append(("shared", 4, full, [128] * ws))
    out.append(("shared", 4, full, [(l % 4) * 4 for l in range(ws)]))
    out.append(("shared", 4, full, [(l // 2) * 128 for l in range(ws)]))
    out.append(("shared", 12, full, [l * 12 + 2 for l in range(ws)]))
    for _ in range(40):
        m = rng.getrandbits(ws) or 1
        w = rng.choice((1, 2, 4, 8, 16))
        out.append(("shared", w, m, [rng.randrange(0, 16384) for _ in _lanes(m)]))
    out.append(("shared", 4, full, [rng.randrange(0, 1 << 20) * 4 for _ in range(ws)]))  # wide rows: host fallback
    # global: coalesced, strided, unaligned line-crossing, random inside / outside the 64-line window
    base = 0x7F1234560000
    for stride in (4, 8, 16, 32, 64, 128, 132, 256):
        for width in (1, 4, 8, 16):
            out.append(("global", width, full, [base + l * stride for l in range(ws)]))
    out.append(("global", 16, full, [base + 120 + l * 16 for l in range(ws)]))
    out.append(("global", 4, full, [base] * ws))
    for _ in range(40):
        m = rng.getrandbits(ws) or 1
        w = rng.choice((1, 2, 4, 8, 16))
        span = rng.choice((512, 4096, 8000, 1 << 20))
        out.append(("global", w, m, [base + rng.randrange(0, span) for _ in _lanes(m)]))
    return out


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
    g = sim.simulate(kl, "QV100", engine="gpu", extra={"-gpu_ingest": "1"})
    c = sim.simulate(kl, "QV100", engine="cpu")
    assert (g.tot_insn, g.tot_cycle) == (c.tot_insn, c.tot_cycle)
    assert "gpu_ingest: shared" in g.output
