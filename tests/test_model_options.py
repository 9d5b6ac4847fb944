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


TRACE_ALL = {"-trace_enabled": "1", "-trace_sampling_core": "-1", "-gpgpu_perf_sim_memcpy": "0",
             "-trace_components": "WARP_SCHEDULER,SCOREBOARD,MEMORY_PARTITION_UNIT,MEMORY_SUBPARTITION_UNIT,"
                                  "INTERCONNECT,LIVENESS"}


def _trace_lines(out):
    return [l for l in out.splitlines() if l.startswith("GPGPU-Sim Cycle ")]


def test_debug_trace_streams(native, traces):
    import re
    base = _run(native, traces["vadd"], {"-gpgpu_perf_sim_memcpy": "0"})
    tr = _run(native, traces["vadd"], TRACE_ALL)
    assert tr.tot_cycle == base.tot_cycle  # tracing never changes timing
    lines = _trace_lines(tr.output)
    streams = {re.match(r"GPGPU-Sim Cycle \d+: (\w+) -", l).group(1) for l in lines}
    assert streams == {"WARP_SCHEDULER", "SCOREBOARD", "MEMORY_PARTITION_UNIT", "MEMORY_SUBPARTITION_UNIT",
                       "INTERCONNECT"}
    cycles = [int(l.split()[2].rstrip(":")) for l in lines]
    assert cycles == sorted(cycles)
    assert "cycles simulated:" in tr.output
    # issue events == warp instructions
    issued = sum(1 for l in lines if "WARP_SCHEDULER" in l)
    m = re.findall(r"gpgpu_n_tot_w_icount = (\d+)", tr.output)
    assert issued == int(m[-1])
    one = _run(native, traces["vadd"], dict(TRACE_ALL, **{"-trace_sampling_core": "3",
                                                          "-trace_components": "WARP_SCHEDULER"}))
    assert {l.split("core ")[1].split()[0] for l in _trace_lines(one.output)} == {"3"}


def test_memlatency_and_visualizer(native, traces, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    s = _run(native, traces["vadd"], {"-gpgpu_memlatency_stat": "14", "-visualizer_enabled": "1",
                                      "-gpgpu_runtime_stat": "500:0", "-gpgpu_perf_sim_memcpy": "0"})
    assert "averagemflatency = " in s.output and "mf_lat_table:" in s.output
    log = open(tmp_path / "gpgpusim_visualizer.log").read().splitlines()
    assert len(log) > 3 and all(l.startswith("kernel=") for l in log)
    assert sum(int(l.split(" insn=")[1].split()[0]) for l in log) == s.tot_insn
    from accel_sim_framework_distributed_amd.plotting import visualizer
    rows = visualizer.parse(str(tmp_path / "gpgpusim_visualizer.log"))
    assert len(rows) == len(log) and len(rows[-1]["sm_insn"]) == 80
    assert "<svg" in visualizer.render(rows)
    # per-unit vectors (AerialVision's per-shader / per-channel views)
    for r in rows:
        assert len(r["sm_l1_miss_rate"]) == 80 and all(0 <= v <= 1 for v in r["sm_l1_miss_rate"])
        assert len(r["ch_dram_util"]) == len(r["ch_l2_hit"]) == len(r["ch_dram_queue"]) > 0
        assert len(r["issue_distro"]) == 3 + 64 and len(r["mf_lat_hist"]) == 16
        # every scheduler cycle lands in exactly one issue bin
        assert sum(visualizer.issue_groups(r["issue_distro"]).values()) == sum(r["issue_distro"])
    # the issued bins count warp instructions (single issue: one per issued cycle)
    issued = sum(sum(r["issue_distro"][3:]) for r in rows)
    assert issued == sum(sum(r["sm_insn"]) for r in rows)
    assert sum(sum(r["mf_lat_hist"]) for r in rows) > 0
    # two-run page, CSV export
    page = visualizer.render(rows, [("again", rows)])
    assert "asim-data" in page and "drawHeat" in page and page.count('"name"') == 2
    csv = visualizer.to_csv(rows, "sm_insn").splitlines()
    assert len(csv) == len(rows) and len(csv[0].split(",")) == 81
    out = tmp_path / "v.html"
    assert visualizer.main([str(tmp_path / "gpgpusim_visualizer.log"), "-o", str(out)]) == 0
    assert out.stat().st_size > 1000
    # gzip logs (the reference's AerialVision input is gzipped) read the same
    import gzip
    gz = tmp_path / "v.log.gz"
    with gzip.open(gz, "wt") as f:
        f.write(open(tmp_path / "gpgpusim_visualizer.log").read())
    assert visualizer.parse(str(gz)) == rows


def test_pipeline_dump(native, traces):
    s = native.Simulator(presets.args_for("QV100", {"-gpgpu_max_cycle": "9000"}) + ["-trace", traces["bfs"]], False)
    s.run()
    d = s.dump_pipeline(-1, 0)
    assert "=== SM " in d and "scoreboard" in d and "=== memory channel 0" in d
    assert "=== memory channel 1" not in d
    assert s.dump_pipeline(-2, -2) == ""


def test_max_cycle_cap_breaks(native, traces):
    s = native.Simulator(presets.args_for("QV100", {"-gpgpu_max_cycle": "3000"}) + ["-trace", traces["bfs"]], False)
    assert s.run() == 0
    assert "break due to reaching the maximum cycles" in s.output
    full = _run(native, traces["bfs"], {})
    assert s.tot_insn < full.tot_insn


def _stat(out, key):
    import re
    m = re.findall(rf"{re.escape(key)} = ([0-9.]+)", out)
    return float(m[-1]) if m else None


def test_instruction_cache(native, traces):
    """-gpgpu_perfect_inst_const_cache 0 routes fetch through the L1I
    (reference shader.cc:918-1020): cold misses cost cycles, every miss is one
    L2 request, and the quiet-cycle skipper stays exact with warps parked in
    imiss_pending."""
    ic = {"-gpgpu_perfect_inst_const_cache": "0"}
    base = _run(native, traces["bfs"], {})
    cold = _run(native, traces["bfs"], ic)
    assert cold.tot_insn == base.tot_insn
    assert cold.tot_cycle > base.tot_cycle
    assert _stat(base.output, "L1I_total_cache_accesses") == 0
    acc = _stat(cold.output, "L1I_total_cache_accesses")
    miss = _stat(cold.output, "L1I_total_cache_misses")
    assert acc > 0 and 0 < miss < acc
    # each SM misses every code line at most once per kernel while it stays resident
    noskip = _run(native, traces["bfs"], dict(ic, **{"-sim_event_skip": "0"}))
    assert (noskip.tot_cycle, noskip.tot_insn) == (cold.tot_cycle, cold.tot_insn)
    # a one-line, one-way cache thrashes
    tiny = _run(native, traces["bfs"], dict(ic, **{"-gpgpu_cache:il1": "N:1:128:1,L:R:f:N:L,S:2:48,4"}))
    assert _stat(tiny.output, "L1I_total_cache_misses") > miss


def test_sqc_invalidate_at_launch(native, traces):
    """-sim_sqc_invalidate_at_launch 1: every kernel starts with cold
    instruction caches (bfs launches the same two kernels repeatedly: the
    misses of later launches come back), exact with and without the quiet-
    cycle skipper; off by default."""
    ic = {"-gpgpu_perfect_inst_const_cache": "0"}
    keep = _run(native, traces["bfs"], ic)
    inv = _run(native, traces["bfs"], dict(ic, **{"-sim_sqc_invalidate_at_launch": "1"}))
    assert inv.tot_insn == keep.tot_insn
    assert _stat(inv.output, "L1I_total_cache_misses") > _stat(keep.output, "L1I_total_cache_misses")
    noskip = _run(native, traces["bfs"], dict(ic, **{"-sim_sqc_invalidate_at_launch": "1", "-sim_event_skip": "0"}))
    assert (noskip.tot_cycle, noskip.tot_insn) == (inv.tot_cycle, inv.tot_insn)


def test_icache_launch_verdict():
    from accel_sim_framework_distributed_amd.hw_stats import icache_launch
    assert icache_launch.verdict([98, 97, 98, 98]) == 1
    assert icache_launch.verdict([98, 0, 0, 0]) == 0


@pytest.mark.slow
def test_dram_write_queue_and_turnaround(native, traces):
    """-dram_seperate_write_queue_enable with <size>:<high>:<low> watermarks
    (reference dram_sched.cc:118-130) and -dram_elimnate_rw_turnaround
    (gpu-sim.h:247-253) change DRAM timing, never the work done.  A small
    write-back L2 makes the kernel evict dirty lines while it streams."""
    small = {"-gpgpu_perf_sim_memcpy": "0", "-gpgpu_cache:dl2": "S:8:128:4,L:B:m:L:P,A:192:4,32:0,32"}
    base = _run(native, traces["vadd"], small)
    assert _stat(base.output, "total dram writes") > 0
    runs = [_run(native, traces["vadd"], dict(small, **x)) for x in (
        {"-dram_seperate_write_queue_enable": "1", "-dram_write_queue_size": "32:28:16"},
        {"-dram_seperate_write_queue_enable": "1", "-dram_write_queue_size": "8:6:2"},
        {"-dram_seperate_write_queue_enable": "1", "-dram_write_queue_size": "8:6:2", "-gpgpu_dram_scheduler": "0"},
        {"-dram_elimnate_rw_turnaround": "1"})]
    for r in runs:
        assert not r.deadlock and r.tot_insn == base.tot_insn
        assert _stat(r.output, "total dram reads") == _stat(base.output, "total dram reads")
    assert runs[1].tot_cycle != base.tot_cycle
    assert runs[3].tot_cycle <= base.tot_cycle


def test_hotspot_backlog_no_loss(native, tmp_path):
    """Every warp of an 80-SM grid stores into the same few lines: one L2
    sub-partition receives far more packets per epoch than its input queue
    holds.  Arrivals wait in the destination's backlog (nothing is dropped,
    no deadlock) and the quiet-cycle skipper stays exact."""
    import numpy as np
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("_Z7hotspotPi", (320, 1, 1), (256, 1, 1), nregs=16)
    for i in range(6):
        k.op("STG.E", [], [4, 5], base=np.full(k.g.nwarps, 0x7000_0000 + 128 * (i % 2), np.int64), stride=0)
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "hot"), [k.build()])
    a = _run(native, kl, {"-gpgpu_perf_sim_memcpy": "0"})
    b = _run(native, kl, {"-gpgpu_perf_sim_memcpy": "0", "-sim_event_skip": "0"})
    assert not a.deadlock
    assert _stat(a.output, "icnt_mem_input_backlog") > 0
    assert "lost to a full backlog ring" not in a.output
    assert (a.tot_cycle, a.tot_insn) == (b.tot_cycle, b.tot_insn)


def test_max_insn_stops_mid_kernel(native, traces):
    """-gpgpu_max_insn is checked every epoch, not only between kernels
    (reference gpgpu_sim::active, gpu-sim.cc:1071-1094): a one-kernel run
    stops within one epoch's worth of issue after the cap."""
    full = _run(native, traces["vadd"], {})
    cap = full.tot_insn // 3
    s = _run(native, traces["vadd"], {"-gpgpu_max_insn": str(cap)})
    assert cap <= s.tot_insn < full.tot_insn
    assert s.tot_cycle < full.tot_cycle
    assert "break due to reaching the maximum" in s.output


def test_max_cta_and_completed_cta_caps(native, traces):
    full = _run(native, traces["vadd"], {})
    n_cta = int(_stat(full.output, "gpu_tot_issued_cta"))
    s = _run(native, traces["vadd"], {"-gpgpu_max_cta": "40"})
    assert int(_stat(s.output, "gpu_tot_issued_cta")) == 40 < n_cta
    assert s.tot_insn < full.tot_insn
    c = _run(native, traces["vadd"], {"-gpgpu_max_completed_cta": "20"})
    assert 20 <= int(_stat(c.output, "gpgpu_n_completed_cta")) < n_cta
    assert c.tot_insn < full.tot_insn


def test_cdna_scalar_loads_use_the_scalar_cache(native, tmp_path):
    """CDNA s_load: an lgkmcnt-counted load through the cache, keyed by kernel
    and code offset (trace.cc coalesce_kernel); the first wave on a CU misses,
    later waves of the same load hit."""
    import re
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder

    def run(smem, ctas, extra):
        k = KernelBuilder("_Z4kargPf", (ctas, 1, 1), (256, 1, 1), nregs=32, binary_version=950, warp_size=64)
        for i in range(8):  # a dependent chain: load, wait, use
            k.op("s_load_dwordx2" if smem else "s_add_u32", [170], [171])
            k.op("s_waitcnt")
            k.op("s_add_u32", [171], [170, 171])
        k.op("v_add_u32", [4], [171, 4])
        k.op("s_endpgm")
        kl = rodinia.write_app(str(tmp_path / f"k{int(smem)}_{ctas}"), [k.build()], memcpy=False)
        s = native.Simulator(presets.args_for("MI355X", dict({"-gpgpu_perf_sim_memcpy": "0"}, **extra))
                             + ["-trace", kl], False)
        assert s.run() == 0
        return s.output

    def stat(out, key):
        return int(re.findall(rf"^{re.escape(key)} = (\d+)", out, re.M)[-1])

    full = run(True, 256, {})
    assert stat(full, "gpgpu_n_load_insn") == 256 * 4 * 8
    # nearby loads share a line (code offset / 8): the chain's 8 loads touch
    # two 32-byte sectors of one 128-byte line, which the MI355X L1 fills
    # whole (line-granular 'N'): one miss per CU (256 CUs, one CTA each); the
    # other accesses hit or merge into it
    l1 = [stat(full, f"\tTotal_core_cache_stats_breakdown[GLOBAL_ACC_R][{k}]") for k in ("HIT", "MISS", "MSHR_HIT")]
    assert l1[1] == 256 and sum(l1) == 256 * 4 * 8
    # latency: eight dependent round trips through the cache on one CU
    quiet = {"-gpgpu_kernel_launch_latency": "0", "-gpgpu_inst_prefetch_lines": "0"}
    ld, alu = run(True, 1, quiet), run(False, 1, quiet)
    assert stat(alu, "gpgpu_n_load_insn") == 0
    assert stat(ld, "gpu_sim_cycle") > stat(alu, "gpu_sim_cycle") + 8 * 100


def test_warp_issue_interval(native, tmp_path):
    """-gpgpu_warp_issue_interval: one warp's independent instructions issue
    at most once per interval (measured on MI355X by ub_wave_issue: ~5.5)."""
    import re
    from accel_sim_framework_distributed_amd.models import presets
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("_Z3ilpPf", (1, 1, 1), (32, 1, 1), nregs=32)
    for i in range(256):
        k.op("FFMA", [8 + i % 8], [8 + i % 8, 4])
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "ilp"), [k.build()], memcpy=False)
    cyc = {}
    for iv in (1, 4):
        s = native.Simulator(presets.args_for("QV100", {"-gpgpu_warp_issue_interval": str(iv),
                                                        "-gpgpu_kernel_launch_latency": "0"}) + ["-trace", kl], False)
        assert s.run() == 0
        cyc[iv] = int(re.findall(r"^gpu_sim_cycle = (\d+)", s.output, re.M)[-1])
    # 256 independent instructions: ~3 extra cycles each
    assert cyc[4] - cyc[1] >= 256 * 2


def test_reply_path_buffers(native, traces):
    """Cluster ejection buffer and LD/ST response FIFO (reference
    simt_core_cluster::icnt_cycle, shader.cc:4623-4660; ldst_unit response
    FIFO, shader.cc:2302-2309,2810-2857): the flags size the two queues every
    reply passes (one extra cycle between the crossbar port and the L1 fill,
    as in the reference's icnt_cycle -> ldst_unit::cycle order); with room for
    one packet each the path still moves one reply per cycle."""
    cfg = native.parse_config(presets.args_for("QV100", {"-gpgpu_n_cluster_ejection_buffer_size": "3",
                                                          "-gpgpu_n_ldst_response_buffer_size": "1"}))
    assert (cfg["eject_buf"], cfg["ldst_resp_buf"]) == (3, 1)
    base = _run(native, traces["vadd"], {})
    tight = _run(native, traces["vadd"], {"-gpgpu_n_cluster_ejection_buffer_size": "1",
                                          "-gpgpu_n_ldst_response_buffer_size": "1"})
    assert tight.tot_insn == base.tot_insn
    assert abs(tight.tot_cycle - base.tot_cycle) <= 0.02 * base.tot_cycle
    # no L1 write-back is ever dropped by a full injection queue
    for r in (base, tight):
        assert "write-backs lost" not in r.output


def test_unmodelled_options_warn(native, traces):
    """Options accepted only for config compatibility never change a run
    silently: a non-default value prints why it has no effect."""
    s = _run(native, traces["vadd"], {"-gpgpu_mem_unit_ports": "2"})
    assert "GPGPU-Sim: WARNING option -gpgpu_mem_unit_ports 2: accepted for config compatibility, not modelled" \
        in s.output
    w = native.unmodelled_option_warnings(presets.args_for("QV100", {}))
    assert not any("ejection_buffer" in x or "response_buffer" in x for x in w)  # both modelled now
    assert any(x.startswith("note: option -gpgpu_ptx_force_max_capability") for x in w)


def test_kernel_launch_model(native, tmp_path):
    """Launch overheads as rocprofv3 sees them on MI355X (ub_launch): a kernel
    queued behind another lasts at least -sim_kernel_min_cycles_queued; with
    a host that submits every -sim_host_launch_interval cycles, kernels that
    arrive after the GPU went idle launch unqueued; the run's first kernel
    pays -sim_first_kernel_latency."""
    kl = rodinia.write_app(str(tmp_path / "p"), rodinia.pathfinder(4000, 12, 2))
    base = _run(native, kl, {})
    ks = [k["cycles"] for k in base.kernels]
    assert len(ks) >= 3
    q = max(ks) * 3
    queued = _run(native, kl, {"-sim_kernel_min_cycles_queued": str(q)})
    kq = [k["cycles"] for k in queued.kernels]
    assert kq[0] == ks[0] and all(c == q for c in kq[1:])
    # a slow host: every kernel finds the GPU idle -> no minimum applies, the
    # gaps are idle time between kernels
    h = q * 4
    slow = _run(native, kl, {"-sim_kernel_min_cycles_queued": str(q), "-sim_host_launch_interval": str(h)})
    assert [k["cycles"] for k in slow.kernels] == ks
    assert slow.tot_cycle >= (len(ks) - 1) * h
    first = _run(native, kl, {"-sim_first_kernel_latency": "777"})
    # (+ at most an epoch: the first CTA dispatch lands on an epoch boundary)
    assert 777 <= first.kernels[0]["cycles"] - ks[0] <= 777 + 32


def test_copy_latency_every_kernel(native, tmp_path):
    """-sim_copy_latency_every_kernel: every kernel launched behind a host copy
    pays -sim_first_kernel_latency (ub_launch measures the after-copy cost on
    each of its copy -> kernel repetitions), not only the run's first."""
    kl = rodinia.write_app(str(tmp_path / "p"), rodinia.pathfinder(4000, 12, 2))
    lines = open(kl).read().splitlines()
    ks = [i for i, l in enumerate(lines) if l.endswith((".traceg", ".asimk", ".traceg.gz"))]
    assert len(ks) >= 3
    # a host copy in front of the second kernel
    lines.insert(ks[1], "MemcpyHtoD,0x7f0000000000,4096")
    open(kl, "w").write("\n".join(lines) + "\n")
    base = _run(native, kl, {"-sim_first_kernel_latency": "777"})
    every = _run(native, kl, {"-sim_first_kernel_latency": "777", "-sim_copy_latency_every_kernel": "1"})
    kb = [k["cycles"] for k in base.kernels]
    ke = [k["cycles"] for k in every.kernels]
    assert ke[0] == kb[0]
    assert 777 <= ke[1] - kb[1] <= 777 + 32
    assert ke[2:] == kb[2:]


def _late_barrier_kernel():
    """One CTA of 4 warps per SM (one warp per scheduler); warps 1-3 reach
    the barrier at once, warp 0 only after a chain of ALU work: the cycle its
    BAR.SYNC issues on scheduler 0 releases the idle schedulers 1-3."""
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    k = KernelBuilder("late_barrier", (80, 1, 1), (128, 1, 1), nregs=16)
    first = k.g.warp == 0
    for _ in range(3):
        k.op("IMAD", [4], [4, 5])
        k.op("BAR.SYNC")
        for _ in range(24):
            k.op("IMAD", [4], [4, 5], present=first)
        k.op("BAR.SYNC")
        k.alu("FFMA", 6)
    k.op("EXIT")
    return k.build()


@pytest.mark.parametrize("app", ["late_barrier", "hotspot", "backprop"])
def test_issue_distro_same_with_scheduler_trace(native, tmp_path, app):
    """The WARP_SCHEDULER trace stream forces the sequential issue loop; the
    lane-parallel one must classify idle schedulers at the same point (after
    the barrier / exit instructions of the schedulers before the first idle
    one), so the warp occupancy distribution is identical with it on and off
    on barrier-heavy kernels."""
    import re
    gen = {"late_barrier": lambda: [_late_barrier_kernel()], "hotspot": lambda: rodinia.hotspot(64, 2, 2),
           "backprop": lambda: rodinia.backprop(1024)}[app]
    kl = rodinia.write_app(str(tmp_path / app), gen())
    off = _run(native, kl, {"-gpgpu_perf_sim_memcpy": "0"})
    on = _run(native, kl, {"-gpgpu_perf_sim_memcpy": "0", "-trace_enabled": "1", "-trace_sampling_core": "5",
                           "-trace_components": "WARP_SCHEDULER"})
    dist = lambda s: re.findall(r"Warp Occupancy Distribution:\n(.*)", s.output)
    assert dist(off) and dist(on) == dist(off)
    assert on.tot_cycle == off.tot_cycle
