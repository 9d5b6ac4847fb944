"""GPU (HIP, gfx950) engine: bit-exact against the CPU reference engine."""
import os
import re

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_mod():
    import torch  # bind torch's HIP runtime first
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    from accel_sim_framework_distributed_amd import _native
    mod = _native.load(prefer_torch_runtime=True)
    assert mod.gpu_available(), "HIP engine cannot see the GPU (native code must run, no silent fallback)"
    return mod


def _both(kl, config="QV100"):
    from accel_sim_framework_distributed_amd import sim
    g = sim.simulate(kl, config, engine="gpu")
    c = sim.simulate(kl, config, engine="cpu")
    return g, c


def test_vectoradd_gpu_equals_cpu(gpu_mod, tmp_path):
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "vadd"), [rodinia.vectoradd()])
    g, c = _both(kl)
    assert g.engine == "gpu" and c.engine == "cpu"
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    strip = lambda s: {k: v for k, v in s.items() if "rate" not in k and "slowdown" not in k and "time" not in k}
    assert strip(g.stats) == strip(c.stats)


@pytest.mark.parametrize("app", ["backprop", "bfs", "nw", "srad_v2"])
def test_rodinia_app_gpu_equals_cpu(gpu_mod, tmp_path, app):
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    gen = {"backprop": lambda: rodinia.backprop(1024), "bfs": lambda: rodinia.bfs(2048, levels=4),
           "nw": lambda: rodinia.nw(64), "srad_v2": lambda: rodinia.srad_v2(64, 64, 1)}[app]
    kl = rodinia.write_app(str(tmp_path / app), gen())
    g, c = _both(kl)
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    assert [k["cycles"] for k in g.kernels] == [k["cycles"] for k in c.kernels]


@pytest.mark.parametrize("extra", [{}, {"-sim_xcd": "8", "-sim_mall": "256:16"}], ids=["shared_l2", "xcd_mall"])
def test_state_snapshot_bit_exact(gpu_mod, tmp_path, extra):
    """Full architectural state (every SM and channel, and the MALL lines) is
    byte-identical."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "hs"), rodinia.hotspot(64, 2, 2))
    sg = sim.Simulator("QV100", kl, engine="gpu", torch_runtime=True, extra=extra)
    sc = sim.Simulator("QV100", kl, engine="cpu", extra=extra)
    sg.run()
    sc.run()
    a, b = sg.native.snapshot(), sc.native.snapshot()
    assert len(a) == len(b)
    assert a == b


@pytest.mark.parametrize("extra", [
    {"-trace_enabled": "1", "-trace_sampling_core": "-1", "-gpgpu_perf_sim_memcpy": "0",
     "-trace_components": "WARP_SCHEDULER,SCOREBOARD,MEMORY_PARTITION_UNIT,MEMORY_SUBPARTITION_UNIT,INTERCONNECT"},
    {"-gpgpu_perfect_mem": "1"},
    {"-gpgpu_simple_dram_model": "1", "-gpgpu_dram_scheduler": "0"},
    {"-sim_event_skip": "0"},
    {"-gpgpu_perfect_inst_const_cache": "0"},
    {"-dram_seperate_write_queue_enable": "1", "-dram_write_queue_size": "16:12:4", "-gpgpu_perf_sim_memcpy": "0"},
    {"-sim_l1_port_bytes": "48", "-sim_l1_addr_lanes_per_cycle": "16"},
    {"-sim_sqc_invalidate_at_launch": "1", "-gpgpu_perfect_inst_const_cache": "0",
     "-sim_l1_port_granule": "32"},
])
def test_model_switches_gpu_equals_cpu(gpu_mod, tmp_path, extra):
    """Debug trace streams (event for event), idealised memory, FIFO DRAM and
    the no-skip path are identical on both engines."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "bfs"), rodinia.bfs(2048, levels=3))
    g = sim.simulate(kl, "QV100", engine="gpu", extra=extra)
    c = sim.simulate(kl, "QV100", engine="cpu", extra=extra)
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    tl = lambda o: [l for l in o.splitlines() if l.startswith("GPGPU-Sim Cycle ")]
    assert tl(g.output) == tl(c.output)


def test_hotspot_backlog_gpu_equals_cpu(gpu_mod, tmp_path):
    """Arrival backlog (more packets per epoch than a sub-partition's input
    queue, both gather paths) is bit-identical on the HIP engine."""
    import numpy as np
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("_Z7hotspotPi", (320, 1, 1), (256, 1, 1), nregs=16)
    for i in range(6):
        k.op("STG.E", [], [4, 5], base=np.full(k.g.nwarps, 0x7000_0000 + 128 * (i % 2), np.int64), stride=0)
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "hot"), [k.build()])
    ex = {"-gpgpu_perf_sim_memcpy": "0"}
    g = sim.simulate(kl, "QV100", engine="gpu", extra=ex)
    c = sim.simulate(kl, "QV100", engine="cpu", extra=ex)
    assert not g.deadlock
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)


@pytest.mark.parametrize("preset", ["TITANX", "GTX480"])
def test_intersim_presets_gpu_equals_cpu(gpu_mod, tmp_path, preset):
    """-network_mode 1 (topology latency per SM/sub-partition pair, lookahead
    from the .icnt router pipeline) is bit-identical on the HIP engine."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "bfs"), rodinia.bfs(2048, levels=3))
    g = sim.simulate(kl, preset, engine="gpu")
    c = sim.simulate(kl, preset, engine="cpu")
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)


def test_engine_kernel_resources(gpu_mod):
    """The persistent engine kernel fits its one-block-per-CU design: the
    dynamic LDS holds the largest unit state, no large scratch, one wavefront."""
    from accel_sim_framework_distributed_amd.ops import engine
    k = engine.kernel_info()
    assert k and k["max_threads_per_block"] >= 64
    assert max(k["sm_state_bytes"], k["chan_state_bytes"]) < k["lds_dynamic"] <= 160 * 1024
    assert k["scratch_bytes_per_lane"] <= 1024
    f = engine.footprint("QV100")
    assert f["blocks"] == 112 and f["concurrent_simulations"] >= 2


def test_check_engine_gpu_vs_cpu_lockstep(gpu_mod, tmp_path):
    """-sim_engine check: GPU and CPU engines run side by side, timing states
    compared byte for byte every 512 cycles (SURVEY §5.2 --check mode)."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.generate_suite(str(tmp_path), ["nw-rodinia-2.0-ft"])["nw-rodinia-2.0-ft"]
    c = sim.simulate(kl, "QV100", engine="cpu")
    k = sim.simulate(kl, "QV100", engine="check", extra={"-sim_check_interval": "512"})
    assert (k.tot_cycle, k.tot_insn) == (c.tot_cycle, c.tot_insn)


# model features added in round 2, each bit-exact on both engines
_FEATURES = {
    "l1_write_back": {"-gpgpu_cache:dl1": "S:4:128:64,L:B:m:L:L,A:512:8,16:0,32"},
    "l1_fetch_on_write": {"-gpgpu_cache:dl1": "S:4:128:64,L:T:m:F:L,A:512:8,16:0,32"},
    "l2_no_write_alloc": {"-gpgpu_cache:dl2": "S:32:128:24,L:B:m:N:P,A:192:4,32:0,32"},
    "dual_issue": {"-gpgpu_max_insn_issue_per_warp": "2"},
    "warp_limiting": {"-gpgpu_scheduler": "warp_limiting:2:2"},
    "two_level": {"-gpgpu_scheduler": "two_level_active:4:0:1"},
    "max_insn_cap": {"-gpgpu_max_insn": "150000"},
    "max_cta_cap": {"-gpgpu_max_cta": "30"},
    "long_epoch": {"-icnt_latency": "32"},
    # round 3: CDNA4 memory hierarchy and the SM reply-path buffers
    "xcd_mall": {"-sim_xcd": "8", "-sim_mall": "256:16", "-sim_mall_miss_latency": "200",
                 "-gpgpu_flush_l2_cache": "1"},
    "reply_buffers": {"-gpgpu_n_cluster_ejection_buffer_size": "1", "-gpgpu_n_ldst_response_buffer_size": "1"},
    # kernel-boundary release into the MALL, line-granular L2 fills, a 2048-line
    # per-channel tag pool (one sub-partition per channel)
    # round-robin CTA -> XCD dispatch, 64 B store requests
    "xcd_dispatch_wr64": {"-sim_xcd": "8", "-sim_l1_write_request_bytes": "64",
                          "-gpgpu_cache:dl1": "S:4:128:64,L:T:m:N:L,A:512:8,16:0,32"},
    "xcd_release_line_l2": {"-sim_xcd": "8", "-sim_mall": "256:16", "-sim_mall_miss_latency": "200",
                            "-sim_l2_kernel_release": "1", "-gpgpu_n_sub_partition_per_mchannel": "1",
                            "-gpgpu_cache:dl2": "N:128:128:16,L:B:m:L:P,A:192:4,32:0,32"},
}


@pytest.mark.parametrize("feature", sorted(_FEATURES))
def test_round2_features_gpu_equals_cpu(gpu_mod, tmp_path, feature):
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "bp"), rodinia.backprop(1024))
    extra = _FEATURES[feature]
    g = sim.simulate(kl, "QV100", engine="gpu", extra=extra)
    c = sim.simulate(kl, "QV100", engine="cpu", extra=extra)
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    strip = lambda s: {k: v for k, v in s.items() if "rate" not in k and "slowdown" not in k and "time" not in k}
    assert strip(g.stats) == strip(c.stats)


def _cdna_stream_kernel():
    """A wave64 gfx950 kernel: 1024 workgroups of 256 threads streaming
    loads/stores through L2/HBM with some VALU and an LDS round trip."""
    import numpy as np
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("k_stream", (1024, 1, 1), (256, 1, 1), nregs=32, binary_version=950, warp_size=64)
    base = k.g.gtid0.astype(np.int64) * 4
    k.op("global_load_dwordx4", [4], [2], base=0x7000_0000 + base * 4, stride=16)
    k.op("global_load_dword", [5], [2], base=0x9000_0000 + base, stride=4)
    k.op("s_waitcnt", [], [])
    k.alu("v_fma_f32", 4, regs=(4, 5, 6))
    k.op("ds_write_b32", [], [4], base=k.g.warp.astype(np.int64) * 256, stride=4)
    k.op("s_barrier")
    k.op("ds_read_b32", [7], [4], base=k.g.warp.astype(np.int64) * 256, stride=4)
    k.op("s_waitcnt", [], [])
    k.op("global_store_dword", [], [7], base=0xB000_0000 + base, stride=4)
    k.op("s_endpgm")
    return k.build()


def test_mi355x_preset_gpu_equals_cpu(gpu_mod, tmp_path):
    """The 384-unit MI355X preset (256 CUs + 128 channels) runs on the HIP
    engine by time-slicing units over the 256 blocks, bit-exact with the CPU."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.ops import engine
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    f = engine.footprint("MI355X")
    assert f["units"] == 384 and f["blocks"] <= f["device_cus"] and f["units_per_block"] >= 2
    kl = rodinia.write_app(str(tmp_path / "cdna"), [_cdna_stream_kernel()])
    g = sim.simulate(kl, "MI355X", engine="gpu")
    c = sim.simulate(kl, "MI355X", engine="cpu")
    assert g.engine == "gpu"
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    strip = lambda s: {k: v for k, v in s.items() if "rate" not in k and "slowdown" not in k and "time" not in k}
    assert strip(g.stats) == strip(c.stats)


@pytest.mark.parametrize("blocks", ["40", "7"])
def test_time_sliced_units_gpu_equals_cpu(gpu_mod, tmp_path, monkeypatch, blocks):
    """QV100 (112 units) squeezed onto 40 / 7 blocks: 3 / 16 units per block,
    SM and channel states swapped through HBM every epoch; still bit-exact."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "hs"), rodinia.hotspot(64, 2, 2))
    c = sim.simulate(kl, "QV100", engine="cpu")
    monkeypatch.setenv("ASIM_GPU_BLOCKS", blocks)
    g = sim.simulate(kl, "QV100", engine="gpu")
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
    assert [k["cycles"] for k in g.kernels] == [k["cycles"] for k in c.kernels]


def test_kernel_without_memory_ops_gpu_equals_cpu(gpu_mod, tmp_path):
    """A kernel with no memory instruction at all (empty access table) runs on
    the HIP engine (regression: the empty table upload used a null host pointer)."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("k_alu", (512, 1, 1), (256, 1, 1), nregs=16, binary_version=950, warp_size=64)
    k.alu("v_fma_f32", 16, regs=(4, 5, 6))
    k.op("s_endpgm")
    kl = rodinia.write_app(str(tmp_path / "alu"), [k.build()], memcpy=False)
    g = sim.simulate(kl, "MI355X", engine="gpu")
    c = sim.simulate(kl, "MI355X", engine="cpu")
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)


def test_power_report_and_dvfs_gpu_equals_cpu(gpu_mod, tmp_path):
    """Power sampling on the MI355X engine: the per-kernel AccelWattch report
    (every component's avg / max / min) and the DVFS governor's clock choices
    are identical to the CPU engine's, sample by sample."""
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.power import report, xmlcfg
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "hs"), rodinia.hotspot(512, 2, 1))
    p = xmlcfg.default_params("QV100")
    xml = str(tmp_path / "aw.xml")
    xmlcfg.write_xml(xml, dict(p, power_cap=150.0, dvfs_v_floor=0.6))
    out = {}
    for eng in ("cpu", "gpu"):
        rep = str(tmp_path / f"p_{eng}.log")
        args = presets.args_for("QV100", {"-power_simulation_enabled": "1", "-accelwattch_xml_file": xml,
                                          "-gpgpu_runtime_stat": "200:0", "-dvfs_enabled": "1",
                                          "-power_report_file": rep, "-sim_engine": eng}) + ["-trace", kl]
        s = gpu_mod.Simulator(args, False)
        assert s.run() == 0
        out[eng] = (s.tot_cycle, report.parse_power_report(rep),
                    [l for l in s.output.splitlines() if l.startswith(("gpu_sim_time_ns", "gpu_avg_core_clock"))])
    assert out["gpu"] == out["cpu"]
    assert out["cpu"][1][0]["kernel_avg_clock_ratio"] < 1.0  # the governor did act


@pytest.mark.parametrize("extra", [{}, {"-sim_xcd": "8", "-sim_mall": "256:16"}], ids=["shared_l2", "xcd_mall"])
def test_trace_window_streaming_gpu_equals_cpu(gpu_mod, tmp_path, extra):
    """-gpu_trace_window: only a window of the kernel's trace (about one
    resident-CTA capacity here) sits in HBM; CTAs stream in as the dispatch
    cursor advances.  Cycles and statistics equal the whole-kernel upload and
    the CPU engine, and the resident trace is a fraction of the kernel's."""
    import numpy as np
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("k_many", (6000, 1, 1), (256, 1, 1), nregs=16)
    base = k.g.gtid0.astype(np.int64) * 4
    k.op("LDG.E", [4], [2], base=0x7000_0000 + base, stride=4)
    k.alu("FFMA", 3, regs=(4, 5, 6))
    k.op("STG.E", [], [2, 4], base=0x9000_0000 + base, stride=4)
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "many"), [k.build()])
    win = sim.simulate(kl, "QV100", engine="gpu", extra=dict(extra, **{"-gpu_trace_window": "1"}))
    whole = sim.simulate(kl, "QV100", engine="gpu", extra=dict(extra, **{"-gpu_trace_window": "0"}))
    cpu = sim.simulate(kl, "QV100", engine="cpu", extra=extra)
    assert (win.tot_cycle, win.tot_insn) == (cpu.tot_cycle, cpu.tot_insn) == (whole.tot_cycle, whole.tot_insn)
    skip = ("rate", "slowdown", "time")
    strip = lambda s: {a: v for a, v in s.items() if not any(x in a for x in skip)}
    assert strip(win.stats) == strip(cpu.stats)
    diag = lambda r, key: int(re.search(key + r": (\d+)", r.output).group(1))
    pw, pf = diag(win, "gpu_trace_resident_peak_bytes"), diag(whole, "gpu_trace_resident_peak_bytes")
    assert diag(win, "gpu_trace_window_fills") > 3
    # the rings are powers of two sized for the oldest resident CTA up to the
    # dispatch bound of the next epochs (XCD round-robin dispatch spreads
    # that span): about 2 K of the 6 K CTAs are resident here
    assert pw * 2 < pf, (pw, pf)


@pytest.mark.parametrize("extra", [{}, {"-sim_xcd": "8", "-sim_mall": "256:16"}], ids=["shared_l2", "xcd_mall"])
def test_host_streamed_trace_gpu_equals_cpu(gpu_mod, tmp_path, extra):
    """-trace_host_budget_mb: the text trace is read per thread block as the
    GPU engine's HBM window advances (host and device windows are the same
    TraceWindows); results equal the CPU engine on the whole kernel."""
    import numpy as np
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("k_many", (6000, 1, 1), (256, 1, 1), nregs=16)
    base = k.g.gtid0.astype(np.int64) * 4
    k.op("LDG.E", [4], [2], base=0x7000_0000 + base, stride=4)
    k.alu("FFMA", 3, regs=(4, 5, 6))
    k.op("STG.E", [], [2, 4], base=0x9000_0000 + base, stride=4)
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "many"), [k.build()], text=True)
    st = sim.simulate(kl, "QV100", engine="gpu",
                      extra=dict(extra, **{"-trace_host_budget_mb": "0.5", "-gpu_trace_window": "1"}))
    cpu = sim.simulate(kl, "QV100", engine="cpu", extra=extra)
    assert (st.tot_cycle, st.tot_insn) == (cpu.tot_cycle, cpu.tot_insn)
    skip = ("rate", "slowdown", "time")
    strip = lambda s: {a: v for a, v in s.items() if not any(x in a for x in skip)}
    assert strip(st.stats) == strip(cpu.stats)
    assert re.search(r"^trace_host_streamed_kernels: 1$", st.output, re.M)


def test_power_in_kernel_gpu_equals_cpu(gpu_mod, tmp_path):
    """Power sampled inside engine_kernel (f64 MFMA sums of every unit's raw
    counters, the sample evaluated by one block into a device ring): the
    report equals the CPU engine's in-loop and host-sliced samples bit for
    bit, and sampling costs no extra kernel launch."""
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.power import xmlcfg
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "hs"), rodinia.hotspot(512, 2, 2))
    xml = str(tmp_path / "aw.xml")
    xmlcfg.write_xml(xml, xmlcfg.default_params("QV100"))
    out = {}
    for tag, eng, inl, pwr in (("gpu", "gpu", "1", "1"), ("cpu", "cpu", "1", "1"), ("cpu_sliced", "cpu", "0", "1"),
                               ("gpu_nopower", "gpu", "1", "0")):
        rep = str(tmp_path / f"p_{tag}.log")
        args = presets.args_for("QV100", {"-power_simulation_enabled": pwr, "-accelwattch_xml_file": xml,
                                          "-gpgpu_runtime_stat": "200:0", "-power_report_file": rep,
                                          "-power_in_loop": inl, "-sim_engine": eng}) + ["-trace", kl]
        s = gpu_mod.Simulator(args, False)
        assert s.run() == 0
        m = re.search(r"^engine_kernel_launches: (\d+)", s.output, re.M)
        n = re.search(r"^power_in_loop_samples: (\d+)", s.output, re.M)
        out[tag] = (s.tot_cycle, open(rep).read() if pwr == "1" else "", int(m.group(1)) if m else 0,
                    int(n.group(1)) if n else 0)
    assert out["gpu"][0] == out["cpu"][0] == out["cpu_sliced"][0] == out["gpu_nopower"][0]
    assert out["gpu"][1] == out["cpu"][1] == out["cpu_sliced"][1] and "kernel_avg_power" in out["gpu"][1]
    assert out["gpu"][3] == out["cpu"][3] >= 10
    # one launch per kernel run either way: sampling does not relaunch
    assert out["gpu"][2] == out["gpu_nopower"][2] > 0


@pytest.mark.parametrize("app", ["bfs", "hotspot"])
def test_global_state_gpu_equals_cpu(gpu_mod, tmp_path, monkeypatch, app):
    """ASIM_GPU_STATE=global: units simulated in place in their HBM images
    (no LDS state, many engine waves per CU) give the CPU engine's full state
    image and statistics, also with fewer blocks than units."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    monkeypatch.setenv("ASIM_GPU_STATE", "global")
    gen = {"bfs": lambda: rodinia.bfs(2048, levels=4), "hotspot": lambda: rodinia.hotspot(64, 2, 2)}[app]
    kl = rodinia.write_app(str(tmp_path / app), gen())
    for blocks in ("0", "37"):
        monkeypatch.setenv("ASIM_GPU_BLOCKS", blocks)
        sg = sim.Simulator("QV100", kl, engine="gpu", torch_runtime=True)
        sc = sim.Simulator("QV100", kl, engine="cpu")
        g, c = sg.run(), sc.run()
        assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
        assert sg.native.snapshot() == sc.native.snapshot()
    # 112 single-wave blocks at several per CU (the kernel's occupancy)
    assert gpu_mod.gpu_cus_per_sim(80, 32) <= 56


def test_device_pool_stays_bounded(gpu_mod, tmp_path):
    """The engine's caching allocator keeps freed buffers for the next
    simulation of the same shape but never caches more than its cap: many
    simulations of different shapes in one process leave the cached bytes
    at or under the cap, and a trim gives everything back."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kl = rodinia.write_app(str(tmp_path / "vadd"), [rodinia.vectoradd(20000)])
    for n in (8, 16, 24, 32, 40, 48, 56, 64):
        sim.simulate(kl, "QV100", engine="gpu", extra={"-gpgpu_n_clusters": str(n)})
        st = gpu_mod.gpu_pool_stats()
        assert st["cached_dev"] <= st["cap_dev"] and st["cached_host"] <= st["cap_host"]
    assert gpu_mod.gpu_pool_stats()["cached_dev"] > 0
    gpu_mod.gpu_pool_trim()
    st = gpu_mod.gpu_pool_stats()
    assert st["cached_dev"] == 0 and st["cached_host"] == 0 and st["trims"] >= 1
    # the engine still works after a trim
    g = sim.simulate(kl, "QV100", engine="gpu")
    c = sim.simulate(kl, "QV100", engine="cpu")
    assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)


@pytest.mark.parametrize("state", ["global", "split"])
def test_batch_launch_many_simulations_gpu_equals_cpu(gpu_mod, tmp_path, monkeypatch, state):
    """Global- / split-state simulations running side by side in one process
    share batch launches (ASIM_GPU_BATCH=1: one launch hosts several
    simulations, each synchronising only its own blocks); every one of them
    stays bit-exact against the CPU engine."""
    from concurrent.futures import ThreadPoolExecutor
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    monkeypatch.setenv("ASIM_GPU_STATE", state)
    monkeypatch.setenv("ASIM_GPU_BATCH", "1")
    apps = {"bfs": rodinia.bfs(2048, levels=3), "hotspot": rodinia.hotspot(64, 2, 2), "nw": rodinia.nw(64),
            "backprop": rodinia.backprop(1024), "srad": rodinia.srad_v2(64, 64, 1), "path": rodinia.pathfinder(2000, 8, 2)}
    kls = {n: rodinia.write_app(str(tmp_path / n), k) for n, k in apps.items()}
    import torch
    dev = torch.cuda.current_device()

    def run_gpu(n):
        torch.cuda.set_device(dev)
        s = sim.Simulator("QV100", kls[n], engine="gpu", torch_runtime=True)
        r = s.run()
        return n, (r.tot_cycle, r.tot_insn), s.native.snapshot()

    before = gpu_mod.gpu_batch_stats()
    with ThreadPoolExecutor(max_workers=len(kls)) as ex:
        got = list(ex.map(run_gpu, list(kls)))
    after = gpu_mod.gpu_batch_stats()
    for n, res, snap in got:
        sc = sim.Simulator("QV100", kls[n], engine="cpu")
        rc = sc.run()
        assert res == (rc.tot_cycle, rc.tot_insn), n
        assert snap == sc.native.snapshot(), n
    launches = after["launches"] - before["launches"]
    batches = after["batches"] - before["batches"]
    assert launches >= len(kls) and batches < launches  # launches were shared


@pytest.mark.parametrize("app", ["bfs", "hotspot"])
def test_split_state_gpu_equals_cpu(gpu_mod, tmp_path, monkeypatch, app):
    """ASIM_GPU_STATE=split: an SM's hot prefix in LDS, its geometry-sized
    arrays (rings, cache tags, MSHRs, pending loads) and every channel in HBM;
    bit-exact against the CPU engine, also time-sliced (37 blocks)."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    monkeypatch.setenv("ASIM_GPU_STATE", "split")
    gen = {"bfs": lambda: rodinia.bfs(2048, levels=4), "hotspot": lambda: rodinia.hotspot(64, 2, 2)}[app]
    kl = rodinia.write_app(str(tmp_path / app), gen())
    for blocks in ("0", "37"):
        monkeypatch.setenv("ASIM_GPU_BLOCKS", blocks)
        sg = sim.Simulator("QV100", kl, engine="gpu", torch_runtime=True)
        sc = sim.Simulator("QV100", kl, engine="cpu")
        g, c = sg.run(), sc.run()
        assert (g.tot_cycle, g.tot_insn) == (c.tot_cycle, c.tot_insn)
        assert sg.native.snapshot() == sc.native.snapshot()


def test_split_state_kernel_resources(gpu_mod):
    """The split-state build needs <= 40 KB of LDS per engine block, so at
    least 4 engine waves share a CU (3 used: one block of margin below the
    occupancy API), and a GV100 simulation (112 units) reserves <= 38 CUs."""
    m = gpu_mod.gpu_engine_modes()
    assert m["split"]["lds_bytes"] <= 40 * 1024
    assert m["split"]["occupancy_api"] >= 4 and m["split"]["blocks_per_cu"] >= 3
    # the hot prefix (instruction window and packet queues in HBM) fits eight
    # blocks' LDS in a CU: the two-waves-per-SIMD kernel reaches 8 per CU
    assert m["split"]["sm_hot_bytes"] <= 17 * 1024 and m["split"]["lds_bytes"] <= 20 * 1024
    assert m["split2"]["occupancy_api"] >= 8
    assert m["lds"]["blocks_per_cu"] == 1 and m["lds"]["lds_bytes"] > m["lds"]["sm_state_bytes"]
    assert gpu_mod.gpu_cus_per_sim(80, 32) <= 38  # split is the default build
