"""Concurrent kernels and the stream window (reference gpu-simulator/main.cc:74-115
window of -gpgpu_max_concurrent_kernel commands with stream-busy gating, and
shader.cc:4502-4535 -gpgpu_concurrent_kernel_sm CTA mixing on one SM), plus
collectives on their own stream overlapping compute."""

import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
from accel_sim_framework_distributed_amd.tracegen.format import write_kernel_binary, write_kernelslist

BASE = 0x7100_0000


def _kernel(kid, stream, ctas=2, threads=64, alu=200, shmem=0, loads=4):
    """`ctas` CTAs of a dependent FFMA chain with a few global loads."""
    k = KernelBuilder(f"_Z2k{kid}Pf", (ctas, 1, 1), (threads, 1, 1), nregs=16, kid=kid, shmem=shmem)
    k.header["stream"] = stream
    g = k.g
    for i in range(loads):
        k.op("LDG.E", [8], [2], base=BASE + kid * (1 << 22) + g.gtid0 * 4 + i * (1 << 16), stride=4)
        k.op("FFMA", [4], [4, 8])
    for _ in range(alu):
        k.op("FFMA", [4], [4, 5])
    k.op("STG.E", [], [2, 4], base=BASE + kid * (1 << 22) + g.gtid0 * 4, stride=4)
    k.op("EXIT")
    return k.build()


def _app(tmp_path, name, kernels, extra_cmds=()):
    d = tmp_path / name
    d.mkdir()
    cmds = []
    for i, k in enumerate(kernels, 1):
        write_kernel_binary(str(d / f"kernel-{i}.asimk"), k)
        cmds.append(f"kernel-{i}.asimk")
    for pos, line in extra_cmds:
        cmds.insert(pos, line)
    return write_kernelslist(str(d), cmds)


def _run(native, kl, conc, extra=None, engine="cpu"):
    over = {"-gpgpu_concurrent_kernel_sm": "1" if conc else "0", "-gpgpu_perf_sim_memcpy": "0",
            "-sim_engine": engine}
    over.update(extra or {})
    s = native.Simulator(presets.args_for("QV100", over) + ["-trace", kl], False)
    assert s.run() == 0
    return s


def test_independent_streams_overlap(native, tmp_path):
    kl = _app(tmp_path, "two", [_kernel(1, 1), _kernel(2, 2)])
    ser = _run(native, kl, False)
    con = _run(native, kl, True)
    ks, kc = ser.kernels, con.kernels
    assert [k["uid"] for k in ks] == [1, 2] and len(kc) == 2
    # serial: kernel 2 starts after kernel 1 ends; concurrent: both start at once
    assert ks[1]["start_cycle"] >= ks[0]["start_cycle"] + ks[0]["cycles"]
    assert kc[0]["start_cycle"] == kc[1]["start_cycle"] == 0
    assert con.tot_cycle < 0.75 * ser.tot_cycle
    assert con.tot_cycle >= max(k["cycles"] for k in ks) * 0.9
    assert con.tot_insn == ser.tot_insn
    assert "launching kernel name: _Z2k2Pf uid: 2" in con.output


def test_same_stream_stays_ordered(native, tmp_path):
    kl = _app(tmp_path, "same", [_kernel(1, 3), _kernel(2, 3)])
    ser = _run(native, kl, False)
    con = _run(native, kl, True)
    # the window holds both, but stream order serialises them exactly
    assert con.tot_cycle == ser.tot_cycle
    assert [k["cycles"] for k in con.kernels] == [k["cycles"] for k in ser.kernels]


def test_kernels_share_one_sm(native, tmp_path):
    # a single SM: with -gpgpu_concurrent_kernel_sm the two kernels' CTAs
    # co-reside (warps / CTA slots permit); the SM then interleaves them
    one = {"-gpgpu_n_clusters": "1"}
    kl = _app(tmp_path, "one_sm", [_kernel(1, 1, ctas=2), _kernel(2, 2, ctas=2)])
    ser = _run(native, kl, False, one)
    con = _run(native, kl, True, one)
    assert con.tot_cycle < 0.8 * ser.tot_cycle
    assert con.tot_insn == ser.tot_insn


def test_shared_memory_limits_mixing(native, tmp_path):
    # each CTA takes 64 KB of the 96 KB shared memory: CTAs of the second
    # kernel cannot join an SM holding one of the first, so one SM runs them
    # back to back even with concurrent kernels enabled
    one = {"-gpgpu_n_clusters": "1", "-gpgpu_shmem_size": "98304", "-gpgpu_adaptive_cache_config": "0",
           "-gpgpu_kernel_launch_latency": "0"}
    kl = _app(tmp_path, "shm", [_kernel(1, 1, ctas=1, shmem=65536), _kernel(2, 2, ctas=1, shmem=65536)])
    ser = _run(native, kl, False, one)
    con = _run(native, kl, True, one)
    k1, k2 = con.kernels
    assert k2["start_cycle"] == 0  # launched at once, but its CTA waits for the SM's shared memory
    assert con.tot_cycle >= 0.95 * ser.tot_cycle
    small = _app(tmp_path, "shm_small", [_kernel(1, 1, ctas=1, shmem=32768), _kernel(2, 2, ctas=1, shmem=32768)])
    assert _run(native, small, True, one).tot_cycle < 0.7 * _run(native, small, False, one).tot_cycle


def test_collective_overlaps_compute_on_its_stream(native, tmp_path):
    # kernel on stream 1, an all-reduce on stream 2, a kernel after it on stream 2
    coll = "ncclAllReduce,count=8388608,dtype=ncclFloat,op=ncclSum,nranks=8,stream=2"
    kl = _app(tmp_path, "coll", [_kernel(1, 1, ctas=8, alu=400), _kernel(2, 2, ctas=8, alu=100)],
              extra_cmds=[(1, coll)])
    extra = {"-collective_model": "ring"}
    ser = _run(native, kl, False, extra)
    con = _run(native, kl, True, extra)
    c = ser.collectives[0]["cycles"]
    assert c > 0 and con.collectives[0]["cycles"] == c
    k1s, k2s = ser.kernels
    k1c, k2c = con.kernels
    # serial: kernel, collective, kernel; concurrent: the collective runs under kernel 1
    assert ser.tot_cycle >= k1s["cycles"] + c
    assert k2c["start_cycle"] >= c and k2c["start_cycle"] < k1s["cycles"] + c
    assert con.tot_cycle < ser.tot_cycle - min(c, k1s["cycles"]) // 2


def test_window_size_bounds_running_kernels(native, tmp_path):
    ks = [_kernel(i, i, ctas=1, alu=100) for i in range(1, 5)]
    kl = _app(tmp_path, "win", ks)
    con2 = _run(native, kl, True, {"-gpgpu_max_concurrent_kernel": "2"})
    starts = sorted(k["start_cycle"] for k in con2.kernels)
    assert starts[0] == starts[1] == 0 and starts[2] > 0
    con4 = _run(native, kl, True, {"-gpgpu_max_concurrent_kernel": "4"})
    assert all(k["start_cycle"] == 0 for k in con4.kernels)
    assert con4.tot_cycle < con2.tot_cycle


@pytest.mark.gpu
def test_concurrent_gpu_matches_cpu(native, tmp_path):
    kl = _app(tmp_path, "gpu", [_kernel(1, 1, ctas=40, alu=150), _kernel(2, 2, ctas=60, alu=80),
                                _kernel(3, 1, ctas=20, alu=50)])
    cpu = _run(native, kl, True)
    gpu = _run(native, kl, True, engine="gpu")
    assert gpu.tot_cycle == cpu.tot_cycle
    assert [(k["uid"], k["start_cycle"], k["cycles"], k["insn"]) for k in gpu.kernels] == \
        [(k["uid"], k["start_cycle"], k["cycles"], k["insn"]) for k in cpu.kernels]


def test_event_orders_streams(native, tmp_path):
    """hipStreamWaitEvent: a kernel on stream 2 that waits for an event
    recorded on stream 1 after kernel 1 starts only when kernel 1 is done."""
    ks = [_kernel(1, 1, ctas=4, alu=200), _kernel(2, 2, ctas=4, alu=100)]
    free = _app(tmp_path, "free", ks)
    dep = _app(tmp_path, "dep", ks, extra_cmds=[(1, "hipEventRecord,event=7,stream=1"),
                                              (2, "hipStreamWaitEvent,stream=2,event=7")])
    a = _run(native, free, True).kernels
    b = _run(native, dep, True).kernels
    assert a[1]["start_cycle"] == 0
    assert b[1]["start_cycle"] >= b[0]["start_cycle"] + b[0]["cycles"]
    # a wait for an event recorded later in the trace does not wait for it
    late = _app(tmp_path, "late", ks, extra_cmds=[(0, "hipStreamWaitEvent,stream=2,event=9"),
                                                 (2, "hipEventRecord,event=9,stream=1")])
    assert _run(native, late, True).kernels[1]["start_cycle"] == 0


def test_trace_prefetch_does_not_change_results(native, tmp_path):
    kl = _app(tmp_path, "pf", [_kernel(i, 1, ctas=3, alu=50) for i in range(1, 5)])
    on = _run(native, kl, False, {"-trace_prefetch": "1"})
    off = _run(native, kl, False, {"-trace_prefetch": "0"})
    assert on.tot_cycle == off.tot_cycle and on.tot_insn == off.tot_insn


def _first_stat(out, key):
    import re
    m = re.findall(rf"{re.escape(key)} = ([0-9.]+)", out)
    return float(m[0]) if m else None


def test_memcpy_behind_kernel_waits_for_it(native, tmp_path):
    """A MemcpyHtoD that follows a kernel in the command list pre-fills the L2
    only after that kernel has been simulated (reference main.cc:83-161 reaches
    the memcpy on the next pass of the command loop).  Kernel 1 reads region R
    cold; the memcpy of R behind it must not turn those reads into L2 hits."""
    region = BASE + 1 * (1 << 22)
    memcpy = f"MemcpyHtoD,0x{region:016x},{1 << 20}"
    kl = _app(tmp_path, "km", [_kernel(1, 0, ctas=4, alu=20), _kernel(2, 0, ctas=4, alu=20)],
              extra_cmds=[(1, memcpy)])
    # reference: the same two kernels with no memcpy at all -> kernel 1 cold
    kl0 = _app(tmp_path, "k0", [_kernel(1, 0, ctas=4, alu=20), _kernel(2, 0, ctas=4, alu=20)])
    for conc in (False, True):
        with_cp = _run(native, kl, conc, {"-gpgpu_perf_sim_memcpy": "1"})
        without = _run(native, kl0, conc, {"-gpgpu_perf_sim_memcpy": "1"})
        key = "L2_cache_stats_breakdown[GLOBAL_ACC_R][HIT]"
        assert _first_stat(with_cp.output, key) == _first_stat(without.output, key)
        assert with_cp.kernels[0]["cycles"] == without.kernels[0]["cycles"]
        # the memcpy lands before kernel 2: its reads of R now hit in the L2
        assert "launching memcpy command" in with_cp.output


def _mem_kernel(kid, stream, ctas=80, loads=24):
    """A memory-bound kernel: every warp streams through its own lines."""
    k = KernelBuilder(f"_Z3mem{kid}Pf", (ctas, 1, 1), (128, 1, 1), nregs=16, kid=kid)
    k.header["stream"] = stream
    g = k.g
    for i in range(loads):
        k.op("LDG.E", [8 + i % 4], [2], base=BASE + kid * (1 << 26) + i * ctas * 512 + g.gtid0 * 4, stride=4)
    for i in range(4):
        k.op("FFMA", [4], [4, 8 + i])
    k.op("EXIT")
    return k.build()


def test_collective_memory_traffic_contends_with_compute(native, tmp_path):
    """-collective_mem_traffic: the all-reduce's send/receive
    buffer traffic runs as an RCCL-style copy kernel through the simulated
    L2 and DRAM.  It adds the ring's 2(n-1)/n x S of reads and writes, and
    slows a memory-bound kernel it overlaps; without overlap the collective
    still completes no earlier than the link model says."""
    coll = "ncclAllReduce,count=2097152,dtype=ncclFloat,op=ncclSum,nranks=8,stream=2"
    kl = _app(tmp_path, "cmem", [_mem_kernel(1, 1)], extra_cmds=[(0, coll)])
    extra = {"-collective_model": "ring"}
    off = _run(native, kl, True, extra)
    on = _run(native, kl, True, dict(extra, **{"-collective_mem_traffic": "1"}))
    assert [k["name"] for k in off.kernels] == ["_Z3mem1Pf"]
    names = [k["name"] for k in on.kernels]
    assert "rccl_AllReduce_copy" in names and "_Z3mem1Pf" in names
    import re

    def tot(out, key):
        return sum(float(x) for x in re.findall(rf"^{re.escape(key)} = ([0-9.]+)", out, re.M)[-1:])
    # 2 (n-1)/n x 8 MiB each way, in 32 B sectors, on top of the kernel's own reads
    moved = 2 * 7 / 8 * 2097152 * 4 / 32
    assert tot(on.output, "L2_to_mem_read_sectors") - tot(off.output, "L2_to_mem_read_sectors") > 0.9 * moved
    comp_off = [k for k in off.kernels if k["name"] == "_Z3mem1Pf"][0]["cycles"]
    comp_on = [k for k in on.kernels if k["name"] == "_Z3mem1Pf"][0]["cycles"]
    assert comp_on > comp_off * 1.05
    assert on.collectives[0]["cycles"] >= off.collectives[0]["cycles"]


@pytest.mark.gpu
def test_collective_memory_traffic_gpu_engine_matches_cpu(native, tmp_path):
    if not native.gpu_available():
        pytest.fail("GPU engine not available on a GPU test run")
    coll = "ncclAllReduce,count=262144,dtype=ncclFloat,op=ncclSum,nranks=4,stream=2"
    kl = _app(tmp_path, "cmemg", [_mem_kernel(1, 1, ctas=16, loads=8)], extra_cmds=[(0, coll)])
    extra = {"-collective_model": "ring", "-collective_mem_traffic": "1"}
    c = _run(native, kl, True, extra)
    g = _run(native, kl, True, extra, engine="gpu")
    assert [(k["name"], k["cycles"]) for k in g.kernels] == [(k["name"], k["cycles"]) for k in c.kernels]
    assert g.tot_cycle == c.tot_cycle
