"""CDNA4 memory hierarchy (MI355X-native extension of the reference's single
address-interleaved L2, l2cache.cc:463-595 / gpu-cache.h:1694): XCD-private L2
slices (-sim_xcd) and the memory-attached Infinity Cache / MALL in front of
every DRAM channel (-sim_mall, -sim_mall_miss_latency)."""
import re

import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
from accel_sim_framework_distributed_amd.tracegen.format import write_kernel_binary, write_kernelslist

BUF = 0x7200_0000
REGION = 32 * 1024          # bytes read by one load instruction over all warps
LOADS = 4                   # load instructions per warp: 128 KB footprint


def _reader(kid, ctas=64):
    """Every warp reads one 128 B line per load; all CTAs sweep the same buffer."""
    k = KernelBuilder(f"_Z4readPf{kid}", (ctas, 1, 1), (128, 1, 1), nregs=16, kid=kid)
    g = k.g
    for i in range(LOADS):
        k.op("LDG.E", [8 + i], [2], base=BUF + i * REGION + (g.gtid0 * 4) % REGION, stride=4)
    for i in range(LOADS):
        k.op("FFMA", [4], [4, 8 + i])
    k.op("EXIT")
    return k.build()


def _shared_reader(kid, ctas=64, loads=16):
    """Every CTA reads the same lines: warp w of any CTA reads line (load, w)."""
    k = KernelBuilder(f"_Z6sharedPf{kid}", (ctas, 1, 1), (128, 1, 1), nregs=16, kid=kid)
    g = k.g
    for i in range(loads):
        k.op("LDG.E", [8], [2], base=BUF + i * 4096 + g.warp * 128, stride=4)
        k.op("FFMA", [4], [4, 8])
    k.op("EXIT")
    return k.build()


def _app(tmp_path, name, nk=1, gen=None):
    d = tmp_path / name
    d.mkdir()
    cmds = []
    for i in range(1, nk + 1):
        write_kernel_binary(str(d / f"kernel-{i}.asimk"), (gen or _reader)(i))
        cmds.append(f"kernel-{i}.asimk")
    return write_kernelslist(str(d), cmds)


def _stat(out, key, first=False):
    m = re.findall(rf"{re.escape(key)} = ([0-9.]+)", out)
    return float(m[0] if first else m[-1]) if m else None


def _run(native, kl, extra, engine="cpu"):
    over = {"-gpgpu_perf_sim_memcpy": "0", "-sim_engine": engine}
    over.update(extra)
    s = native.Simulator(presets.args_for("QV100", over) + ["-trace", kl], False)
    assert s.run() == 0
    return s


def test_config_validation(native):
    cfg = native.parse_config(presets.args_for("QV100", {"-sim_xcd": "8", "-sim_mall": "256:16"}))
    assert cfg["n_sm"] == 80
    with pytest.raises(Exception, match="sim_xcd"):
        native.parse_config(presets.args_for("QV100", {"-sim_xcd": "3"}))
    with pytest.raises(Exception, match="sim_mall"):
        native.parse_config(presets.args_for("QV100", {"-sim_mall": "100:16"}))


def test_xcd_private_l2_replicates_shared_data(native, tmp_path):
    kl = _app(tmp_path, "one", gen=_shared_reader)
    shared = _run(native, kl, {})
    xcd = _run(native, kl, {"-sim_xcd": "8"})
    assert xcd.tot_insn == shared.tot_insn
    lines = 16 * 4
    rd_shared = _stat(shared.output, "L2_to_mem_read_sectors")
    rd_xcd = _stat(xcd.output, "L2_to_mem_read_sectors")
    # one shared L2 fetches every sector once; eight private ones each fetch it
    assert rd_shared == pytest.approx(4 * lines, rel=0.02)
    assert rd_xcd == pytest.approx(8 * 4 * lines, rel=0.05)
    assert "XCDs = 8 (private L2 slices per XCD = 8)" in xcd.output


def test_mall_serves_rereads_after_l2_flush(native, tmp_path):
    kl = _app(tmp_path, "two", nk=2)
    flush = {"-gpgpu_flush_l2_cache": "1", "-sim_mall_miss_latency": "300"}
    no_mall = _run(native, kl, flush)
    mall = _run(native, kl, dict(flush, **{"-sim_mall": "512:16"}))
    sectors = LOADS * REGION // 32
    # kernel 2 re-reads everything: without the MALL from DRAM again
    assert _stat(no_mall.output, "total dram reads") == pytest.approx(2 * sectors, rel=0.02)
    assert _stat(mall.output, "total dram reads") == pytest.approx(sectors, rel=0.02)
    assert _stat(mall.output, "MALL_read_hits") == pytest.approx(sectors, rel=0.02)
    assert _stat(mall.output, "L2_to_mem_read_sectors") == _stat(no_mall.output, "L2_to_mem_read_sectors")
    # the second kernel's misses return at MALL latency: faster than the first
    k1, k2 = mall.kernels
    assert k2["cycles"] < k1["cycles"]


def test_mall_absorbs_writes(native, tmp_path):
    """Stores write back into the MALL (write-allocate): DRAM sees only its
    dirty evictions, and a later reader of the data hits there."""
    k = KernelBuilder("_Z5writePf", (64, 1, 1), (128, 1, 1), nregs=16, kid=1)
    g = k.g
    for i in range(LOADS):
        k.op("STG.E", [], [2, 4], base=BUF + i * REGION + (g.gtid0 * 4) % REGION, stride=4)
    k.op("EXIT")
    d = tmp_path / "w"
    d.mkdir()
    write_kernel_binary(str(d / "kernel-1.asimk"), k.build())
    write_kernel_binary(str(d / "kernel-2.asimk"), _reader(2))
    kl = write_kernelslist(str(d), ["kernel-1.asimk", "kernel-2.asimk"])
    # a write-through L2 sends every store below it; the flush makes the
    # reader miss in the L2
    wt = {"-gpgpu_cache:dl2": "S:32:128:24,L:T:m:L:P,A:192:4,32:0,32", "-gpgpu_flush_l2_cache": "1"}
    base = _run(native, kl, wt)
    mall = _run(native, kl, dict(wt, **{"-sim_mall": "512:16"}))
    sectors = LOADS * REGION // 32
    assert _stat(base.output, "total dram writes") > 0
    assert _stat(base.output, "total dram reads") == pytest.approx(sectors, rel=0.02)
    assert _stat(mall.output, "total dram writes") == 0
    assert _stat(mall.output, "MALL_writes") == _stat(mall.output, "L2_to_mem_write_sectors") > 0
    assert _stat(mall.output, "total dram reads") == 0
    assert _stat(mall.output, "MALL_read_hits") == pytest.approx(sectors, rel=0.02)


def _writer_then_reader(tmp_path):
    k = KernelBuilder("_Z5writePf", (64, 1, 1), (128, 1, 1), nregs=16, kid=1)
    g = k.g
    for i in range(LOADS):
        k.op("STG.E", [], [2, 4], base=BUF + i * REGION + (g.gtid0 * 4) % REGION, stride=4)
    k.op("EXIT")
    d = tmp_path / "rel"
    d.mkdir()
    write_kernel_binary(str(d / "kernel-1.asimk"), k.build())
    write_kernel_binary(str(d / "kernel-2.asimk"), _reader(2))
    return write_kernelslist(str(d), ["kernel-1.asimk", "kernel-2.asimk"])


def test_kernel_release_writes_back_and_invalidates(native, tmp_path):
    """-sim_l2_kernel_release: the end-of-kernel release of a multi-XCD GPU
    writes the dirty L2 sectors to the MALL and the next kernel starts with
    cold L2s (it re-reads from the MALL, DRAM sees nothing)."""
    kl = _writer_then_reader(tmp_path)
    wb = {"-gpgpu_cache:dl2": "S:32:128:24,L:B:m:L:P,A:192:4,32:0,32", "-sim_mall": "512:16"}
    keep = _run(native, kl, wb)
    rel = _run(native, kl, dict(wb, **{"-sim_l2_kernel_release": "1"}))
    sectors = LOADS * REGION // 32
    # without the release the stores stay dirty in the L2 and the reader hits
    assert _stat(keep.output, "L2_to_mem_write_sectors") == 0
    assert _stat(keep.output, "L2_to_mem_read_sectors") == 0
    # with it: every dirty sector goes to the MALL once, the reader misses the
    # L2 and hits the MALL
    assert _stat(rel.output, "L2_to_mem_write_sectors") == pytest.approx(sectors, rel=0.02)
    assert _stat(rel.output, "L2_cache_dirty_evictions") == pytest.approx(sectors / 4, rel=0.02)
    assert _stat(rel.output, "MALL_writes") == _stat(rel.output, "L2_to_mem_write_sectors")
    assert _stat(rel.output, "MALL_read_hits") == pytest.approx(sectors, rel=0.02)
    assert _stat(rel.output, "total dram reads") == 0 and _stat(rel.output, "total dram writes") == 0


def test_line_granular_l2_fetches_whole_lines(native, tmp_path):
    """An 'N' (non-sectored) L2 fetches every sector of a missing line (the
    MI355X L2's 128 B fills, TCC_EA0_RDREQ_128B); a sectored one only what was
    asked for."""
    k = KernelBuilder("_Z5sparsePf", (64, 1, 1), (32, 1, 1), nregs=16, kid=1)
    g = k.g
    # each warp reads ONE sector (every lane the same word) of its own line
    k.op("LDG.E", [8], [2], base=BUF + g.cta * 128, stride=0)
    k.op("EXIT")
    d = tmp_path / "sp"
    d.mkdir()
    write_kernel_binary(str(d / "kernel-1.asimk"), k.build())
    kl = write_kernelslist(str(d), ["kernel-1.asimk"])
    sect = _run(native, kl, {"-gpgpu_cache:dl2": "S:32:128:24,L:B:m:L:P,A:192:4,32:0,32"})
    line = _run(native, kl, {"-gpgpu_cache:dl2": "N:32:128:24,L:B:m:L:P,A:192:4,32:0,32"})
    assert _stat(sect.output, "L2_to_mem_read_sectors") == 64
    assert _stat(line.output, "L2_to_mem_read_sectors") == 4 * 64



def test_xcd_round_robin_cta_dispatch_and_64b_stores(native, tmp_path):
    """-sim_xcd: CTA i runs on an SM of XCD i % n_xcd (the hardware's
    workgroup round robin), so a CTA's lines stay in one XCD's L2 however the
    SMs free up; -sim_l1_write_request_bytes 64 sends a full-line store as two
    L2 write requests."""
    k = KernelBuilder("_Z5storePf", (64, 1, 1), (128, 1, 1), nregs=16, kid=1)
    g = k.g
    # each warp stores one whole 128 B line
    k.op("STG.E", [], [2, 4], base=BUF + g.gtid0 * 4, stride=4)
    k.op("EXIT")
    d = tmp_path / "st"
    d.mkdir()
    write_kernel_binary(str(d / "kernel-1.asimk"), k.build())
    kl = write_kernelslist(str(d), ["kernel-1.asimk"])
    base = {"-sim_xcd": "8"}
    one = _run(native, kl, base)
    two = _run(native, kl, dict(base, **{"-sim_l1_write_request_bytes": "64"}))
    w1 = _stat(one.output, "L2_cache_stats_breakdown[GLOBAL_ACC_W][TOTAL_ACCESS]")
    w2 = _stat(two.output, "L2_cache_stats_breakdown[GLOBAL_ACC_W][TOTAL_ACCESS]")
    assert w1 == 64 * 4 and w2 == 2 * w1
    assert one.tot_insn == two.tot_insn
    with pytest.raises(Exception, match="sim_xcd"):
        native.parse_config(presets.args_for("QV100", {"-sim_xcd": "32", "-gpgpu_n_clusters": "8"}))


def test_l1_64b_tag_lookups(native, tmp_path):
    # one 128 B line per warp load, both 64 B halves: two TCP-style lookups
    kl = _app(tmp_path, "lk")
    s = _run(native, kl, {})
    warps = 64 * 4
    assert _stat(s.output, "L1D_total_64B_tag_lookups") == warps * LOADS * 2


def test_instruction_fetch_blocks(native, tmp_path):
    # 16-byte trace instructions: a 64 B fetch block holds four, so the L1I is
    # read once per block a warp enters (9 instructions = 3 blocks, plus the
    # re-reads after a miss) instead of once per two-instruction fetch; hits
    # cost nothing, so the timing is unchanged
    kl = _app(tmp_path, "ifb")
    base = {"-gpgpu_perfect_inst_const_cache": "0"}
    probe = _run(native, kl, base)
    blk = _run(native, kl, dict(base, **{"-gpgpu_inst_fetch_block_bytes": "64"}))
    a0, a1 = _stat(probe.output, "L1I_total_cache_accesses"), _stat(blk.output, "L1I_total_cache_accesses")
    assert a0 > 0 and a1 > 0
    warps = 64 * 4
    assert warps * 3 <= a1 < a0
    assert _stat(blk.output, "L1I_total_cache_misses") == _stat(probe.output, "L1I_total_cache_misses")
    assert blk.tot_cycle == probe.tot_cycle
    with pytest.raises(Exception, match="power of two"):
        native.parse_config(presets.args_for("QV100", {"-gpgpu_inst_fetch_block_bytes": "48"}))
