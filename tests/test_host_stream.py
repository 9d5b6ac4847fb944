"""Host-side per-CTA trace streaming (-trace_host_budget_mb): a text kernel
trace larger than the budget is read one thread block at a time as the
engine's trace window advances, so the host holds the window, not the kernel
(reference: thread blocks are parsed from the file as CTAs issue,
gpu-simulator/trace-parser/trace_parser.cc:387-447).  Results are bit-exact
with the whole-kernel load on the CPU engine; the GPU engine case is in
tests/test_gpu_engine.py."""
import random
import re

import numpy as np
import pytest


def _kernel(n_cta=6000, name="k_many"):
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder(name, (n_cta, 1, 1), (256, 1, 1), nregs=16)
    base = k.g.gtid0.astype(np.int64) * 4
    k.op("LDG.E", [4], [2], base=0x7000_0000 + base, stride=4)
    k.alu("FFMA", 3, regs=(4, 5, 6))
    k.op("STG.E", [], [2, 4], base=0x9000_0000 + base, stride=4)
    k.op("EXIT")
    return k.build()


@pytest.fixture(scope="module")
def text_app(tmp_path_factory):
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    d = tmp_path_factory.mktemp("hs")
    return rodinia.write_app(str(d / "many"), [_kernel()], text=True)


def _kernel_file(kl):
    import os
    return os.path.join(os.path.dirname(kl), "kernel-1.traceg")


def _shuffled_copy(src, dst, drop=None, seed=1):
    """the same trace with its thread blocks in a random file order (and one
    optionally left out: an empty CTA)"""
    text = open(src).read()
    head, _, body = text.partition("#BEGIN_TB")
    blocks = ["#BEGIN_TB" + b for b in body.split("#BEGIN_TB")]
    random.Random(seed).shuffle(blocks)
    if drop is not None:
        blocks = [b for b in blocks if f"thread block = {drop},0,0\n" not in b]
    open(dst, "w").write(head + "".join(blocks))


def _args():
    from accel_sim_framework_distributed_amd.models import presets
    return presets.args_for("QV100", {})


@pytest.mark.parametrize("step", [1, 37, 640])
def test_reader_equals_whole_load(text_app, step):
    from accel_sim_framework_distributed_amd import _native
    d = _native.load().stream_compare(_kernel_file(text_app), _args(), step)
    assert d["equal"], d
    # at most `step` CTAs resident (plus vector slack): a fraction of the kernel
    if step <= 640:
        assert d["stream_peak_bytes"] * 4 < d["whole_bytes"], d


def test_reader_out_of_order_and_missing_blocks(text_app, tmp_path):
    """thread blocks out of linear order (the reader indexes the file once and
    seeks) and a block missing from the file (an empty CTA, as the whole load)"""
    from accel_sim_framework_distributed_amd import _native
    p = str(tmp_path / "kernel-1.traceg")
    _shuffled_copy(_kernel_file(text_app), p, drop=123)
    d = _native.load().stream_compare(p, _args(), 50)
    assert d["equal"], d


def _strip(s):
    skip = ("rate", "slowdown", "time")
    return {a: v for a, v in s.items() if not any(x in a for x in skip)}


def _diag(r, key):
    m = re.search("^" + key + r": (\d+)", r.output, re.M)
    return int(m.group(1)) if m else None


@pytest.mark.slow
@pytest.mark.parametrize("extra", [{}, {"-sim_xcd": "8", "-sim_mall": "256:16"}], ids=["shared_l2", "xcd_mall"])
def test_cpu_engine_streamed_equals_whole(text_app, extra):
    from accel_sim_framework_distributed_amd import _native, sim
    whole = sim.simulate(text_app, "QV100", engine="cpu", extra=extra)
    st = sim.simulate(text_app, "QV100", engine="cpu",
                      extra=dict(extra, **{"-trace_host_budget_mb": "0.5", "-gpu_trace_window": "1"}))
    assert (st.tot_cycle, st.tot_insn) == (whole.tot_cycle, whole.tot_insn)
    assert _strip(st.stats) == _strip(whole.stats)
    assert _diag(whole, "trace_host_streamed_kernels") is None
    assert _diag(st, "trace_host_streamed_kernels") == 1
    # host trace bytes: the window, a fraction of the whole decoded kernel
    wb = _native.load().stream_compare(_kernel_file(text_app), _args(), 1 << 30)["whole_bytes"]
    peak = _diag(st, "trace_host_peak_bytes")
    assert peak and peak * 2 < wb, (peak, wb)
    assert _diag(st, "gpu_trace_window_fills") > 3


def test_budget_above_file_size_loads_whole(text_app):
    from accel_sim_framework_distributed_amd import sim
    r = sim.simulate(text_app, "QV100", engine="cpu", extra={"-trace_host_budget_mb": "1024"})
    assert _diag(r, "trace_host_streamed_kernels") is None


def test_streamed_shuffled_trace_simulates_identically(text_app, tmp_path):
    """a trace whose thread blocks are out of order streams through the index
    path and still simulates bit-exactly"""
    import os
    import shutil
    from accel_sim_framework_distributed_amd import sim
    d = tmp_path / "shuf"
    d.mkdir()
    shutil.copy(text_app, d / "kernelslist.g")
    _shuffled_copy(_kernel_file(text_app), str(d / "kernel-1.traceg"))
    kl = str(d / "kernelslist.g")
    assert os.path.exists(d / "kernel-1.traceg")
    a = sim.simulate(text_app, "QV100", engine="cpu")
    b = sim.simulate(kl, "QV100", engine="cpu", extra={"-trace_host_budget_mb": "0.5", "-gpu_trace_window": "1"})
    assert (a.tot_cycle, a.tot_insn) == (b.tot_cycle, b.tot_insn)
    assert _strip(a.stats) == _strip(b.stats)


@pytest.mark.slow
@pytest.mark.timeout(120)
def test_malformed_streamed_trace_fails_cleanly_with_thread_team(text_app, tmp_path):
    """a streamed trace whose late thread block names a warp outside its block
    raises from the reader inside the CPU engine's thread team: the run must
    end with that error on every thread count (the team used to
    hang at its barrier with the exception in flight)"""
    import shutil
    from accel_sim_framework_distributed_amd import sim
    d = tmp_path / "bad"
    d.mkdir()
    shutil.copy(text_app, d / "kernelslist.g")
    text = open(_kernel_file(text_app)).read()
    i = text.index("thread block = 5000,0,0\n")
    j = text.index("warp = 3\n", i)
    open(d / "kernel-1.traceg", "w").write(text[:j] + "warp = 99\n" + text[j + len("warp = 3\n"):])
    kl = str(d / "kernelslist.g")
    for thr in ("1", "4"):
        with pytest.raises(Exception, match="warp id outside block"):
            sim.simulate(kl, "QV100", engine="cpu", extra={"-trace_host_budget_mb": "0.5", "-gpu_trace_window": "1",
                                                           "-sim_cpu_threads": thr})
