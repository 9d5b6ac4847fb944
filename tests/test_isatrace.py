"""Automatic gfx950 ISA tracer (isatrace): assembly rewriting on the CPU,
capture + simulation on the MI355X."""
import os
import re
import shutil
import subprocess

import pytest

from accel_sim_framework_distributed_amd.isatrace import rewrite, verify

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_ASM = """	.amdgcn_target "amdgcn-amd-amdhsa--gfx950"
	.text
	.globl	k
	.p2align	8
	.type	k,@function
k:
; %bb.0:
	s_load_dwordx4 s[4:7], s[0:1], 0x0
	v_cmp_gt_i32_e32 vcc, 5, v0
	s_and_saveexec_b64 s[2:3], vcc
	s_cbranch_execz .LBB0_2
; %bb.1:
	s_waitcnt lgkmcnt(0)
	global_load_dword v1, v0, s[4:5] offset:16
	ds_read2_b32 v[2:3], v4 offset0:1 offset1:18
	buffer_store_dword v1, v0, s[4:7], 0 offen offset:8
	global_atomic_add v5, v[6:7], v1, off sc0
.LBB0_2:
	s_or_b64 exec, exec, s[2:3]
	s_endpgm
	.section	.rodata,"a",@progbits
	.p2align	6, 0x0
	.amdhsa_kernel k
		.amdhsa_group_segment_fixed_size 256
		.amdhsa_user_sgpr_count 2
		.amdhsa_user_sgpr_kernarg_segment_ptr 1
		.amdhsa_system_sgpr_workgroup_id_x 1
		.amdhsa_system_sgpr_workgroup_id_y 0
		.amdhsa_system_sgpr_workgroup_id_z 0
		.amdhsa_system_vgpr_workitem_id 0
		.amdhsa_next_free_vgpr 8
		.amdhsa_next_free_sgpr 8
		.amdhsa_accum_offset 8
	.end_amdhsa_kernel
	.text
.Lfunc_end0:
	.size	k, .Lfunc_end0-k
"""


def test_segments_and_memory_ops():
    lines = _ASM.split("\n")
    ks = rewrite.parse_kernels(lines)
    k = ks["k"]
    rewrite.segment(k, lines)
    mn = [i.mnem for i in k.insts]
    assert mn[0] == "s_load_dwordx4" and mn[-1] == "s_endpgm"
    # segment cuts: after the EXEC write (saveexec), after the branch, at the
    # label, after s_or_b64 exec
    segs = [[k.insts[i].mnem for i in s] for s in k.segments]
    assert segs[0][-1] == "s_and_saveexec_b64"
    assert segs[1] == ["s_cbranch_execz"]
    assert segs[2][0] == "s_waitcnt" and segs[2][-1] == "global_atomic_add"
    assert segs[3] == ["s_or_b64"] and segs[4] == ["s_endpgm"]
    mems = [(i.mnem, i.mem_id) for i in k.insts if i.mem_id >= 0]
    assert mems == [("global_load_dword", 0), ("ds_read2_b32", 1), ("buffer_store_dword", 2),
                    ("global_atomic_add", 3)]
    # trace registers: destination tuples, sources; returning atomics have a dst
    d = {i.mnem: rewrite.reg_operands(i) for i in k.insts}
    assert d["ds_read2_b32"] == (["v2", "v3"], ["v4"])
    assert d["buffer_store_dword"] == ([], ["v1", "v0", "s4"])
    assert d["global_atomic_add"] == (["v5"], ["v6", "v1"])
    assert d["v_cmp_gt_i32_e32"][0] == []


def test_instrumented_asm_keeps_program_and_reserves_registers():
    new, maps = rewrite.instrument(_ASM)
    km = maps[0]
    assert km.name == "k" and km.n_mem == 4 and len(km.segments) == 5 and km.lds == 256 and km.vgprs == 8
    # every original instruction survives, in order
    orig = [l.strip() for l in _ASM.split("\n") if rewrite.split_inst(l)]
    body = [l.strip() for l in new.split("\n")]
    at = body.index("k:")
    for o in orig:  # found in order after the previous one
        at = body.index(o, at + 1)
    # probe registers above the kernel's own: s8..s23, v8..v15; descriptor raised
    assert ".amdhsa_next_free_sgpr 24" in new and ".amdhsa_next_free_vgpr 16" in new
    assert ".amdhsa_system_sgpr_workgroup_id_z 1" in new and ".amdhsa_system_vgpr_workitem_id 2" in new
    used = {int(x) for x in re.findall(r"\bs(\d+)\b", new.split(".amdhsa_kernel")[0].split("k:")[1])}
    assert max(used) <= 23
    # the probes' control block is a protected device global
    assert "__asim_tctl:" in new and ".protected\t__asim_tctl" in new
    # address of the saddr global load: v0 + s[4:5] + 16
    at = new.index("global_load_dword v1, v0")
    blk = new[new.rindex("_ret_", 0, at):at]
    assert "v_add_co_u32_e64 v8, s[14:15], s4, v8" in blk and "s_mov_b32 s17, 0x10" in blk
    # map: segment/instruction lines in trace order (ndst dsts mnemonic nsrc srcs width)
    m = rewrite.write_map(maps)
    assert m.startswith(f"ASIMISA 1 {rewrite.CHUNK_UNITS}\nK k 5 4 256 8\nS 1 3\n")
    assert "0 1 2 v2 v3 ds_read2_b32 1 v4 4" in m


def test_probe_spin_limit_comes_from_the_control_block():
    """A wave waiting for a ring slot polls at most ctl.spin_limit times (the
    host sets it; the compiled default only when it is 0), then stops
    recording -- which the host turns into a failed capture."""
    new, _ = rewrite.instrument(_ASM)
    blk = new[new.index("_take_"):new.index("_got_")]
    assert ", 0x18" in blk and "s_load_dword" in blk
    assert "s_cselect_b32" in blk
    assert f"{rewrite.SPIN_LIMIT:#x}" in blk


def test_verify_classes_and_trace_counts(tmp_path):
    assert verify.classify("v_mfma_f32_32x32x16_bf16") == "VALU"
    assert verify.classify("s_load_dwordx2") == "SMEM"
    assert verify.classify("s_cbranch_execz") == "BRANCH"
    assert verify.classify("s_waitcnt") == "OTHER" and verify.classify("s_and_b32") == "SALU"
    assert verify.classify("global_atomic_add") == "VMEM_RD" and verify.classify("buffer_store_dword") == "VMEM_WR"
    t = tmp_path / "kernel-1.traceg"
    t.write_text("-kernel name = k\n\n#BEGIN_TB\n\nthread block = 0,0,0\n\nwarp = 0\ninsts = 3\n"
                 "0000 ffffffffffffffff 1 s3 s_load_dword 1 s0 0\n"
                 "0008 ffffffffffffffff 2 v6 v7 global_load_dwordx2 1 v4 8 0 0x10 0x18\n"
                 "0010 0000000000000003 0 s_endpgm 0 0\n\n#END_TB\n")
    c = verify.trace_counts(str(t))
    assert c["WAVES"] == 1 and c["SMEM"] == 1 and c["VMEM_RD"] == 1 and c["OTHER"] == 1


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc (cross-compiles gfx950 without a GPU)")
def test_rewrite_assembles_for_every_app(tmp_path):
    """The real gfx950 assembly of every suite app instruments and assembles."""
    from accel_sim_framework_distributed_amd.isatrace import build
    for app in ("hotspot", "bfs"):
        fb, maps = build.instrument_source(os.path.join(ROOT, "csrc", "apps", f"{app}.hip"), str(tmp_path),
                                           ["-munsafe-fp-atomics", f"-I{ROOT}/csrc"])
        assert os.path.getsize(fb) > 0 and maps and all(m.n_mem > 0 for m in maps)
        # real byte offsets (4- and 8-byte encodings) from the disassembly
        pcs = [i.pc for i in maps[0].insts]
        assert pcs == sorted(pcs) and len(set(pcs)) == len(pcs) and any(b - a == 8 for a, b in zip(pcs, pcs[1:]))


@pytest.mark.gpu
def test_isatrace_capture_matches_simulation(tmp_path):
    """The instrumented vectoradd computes the right answer, traces one wave
    per 64 threads, and the simulator replays exactly the traced instructions."""
    exe = os.path.join(ROOT, "bin", "isatrace", "vectoradd")
    assert os.path.exists(exe), "build_native.py builds bin/isatrace/*"
    env = dict(os.environ, ASIM_TRACE_DIR=str(tmp_path), ASIM_TRACE_BUF_MB="512")
    r = subprocess.run([exe, "16384"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    kl = tmp_path / "kernelslist.g"
    lines = kl.read_text().split("\n")
    assert lines[0].startswith("MemcpyHtoD,") and "kernel-1.traceg" in lines
    c = verify.trace_counts(str(tmp_path / "kernel-1.traceg"))
    assert c["WAVES"] == 16384 // 64 and c["VMEM_RD"] == 2 * 256 and c["VMEM_WR"] == 256
    from accel_sim_framework_distributed_amd import sim
    s = sim.simulate(str(kl), "MI355X", engine="gpu")
    assert s.stats["gpgpu_n_tot_w_icount"] == sum(v for k, v in c.items() if k != "WAVES")
    assert s.tot_insn == 16384 * (sum(v for k, v in c.items() if k != "WAVES") // 256)


def _trace_body(path):
    """kernel-N.traceg without the header lines (the per-CTA / per-wave part),
    each line's lane addresses as offsets from its first lane's (the two
    captures run as separate processes, whose allocations may sit at
    different addresses)"""
    txt = open(path).read()
    out = []
    for ln in txt[txt.index("#BEGIN_TB"):].split("\n"):
        toks = ln.split()
        addrs = [int(t, 16) for t in toks if t.startswith("0x")]
        if addrs:
            ln = " ".join(t for t in toks if not t.startswith("0x")) + " " + " ".join(str(a - addrs[0]) for a in addrs)
        out.append(ln)
    return "\n".join(out)


@pytest.mark.gpu
def test_isatrace_ring_streams_a_trace_larger_than_the_ring(tmp_path):
    """Streaming capture: vectoradd's 4096 waves need 4096 chunks (32 MB of
    records) and go through a 1 MB host ring (128 slots) drained while the
    kernel runs; the trace equals the one captured into a device buffer that
    holds it whole, nothing is dropped, and it simulates."""
    exe = os.path.join(ROOT, "bin", "isatrace", "vectoradd")
    assert os.path.exists(exe), "build_native.py builds bin/isatrace/*"
    n = 1 << 18
    ring, whole = tmp_path / "ring", tmp_path / "whole"
    env = {k: v for k, v in os.environ.items() if not k.startswith("ASIM_TRACE")}
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(ring), ASIM_TRACE_RING_MB="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    assert "dropped" not in r.stderr and "out of sequence" not in r.stderr, r.stderr
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(whole), ASIM_TRACE_BUF_MB="256"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    c = verify.trace_counts(str(ring / "kernel-1.traceg"))
    assert c["WAVES"] == n // 64 and c["VMEM_WR"] == n // 64
    assert _trace_body(ring / "kernel-1.traceg") == _trace_body(whole / "kernel-1.traceg")
    # spill files are removed once the kernel's trace is written
    assert not [p for p in os.listdir(ring) if p.endswith(".chunks")]
    from accel_sim_framework_distributed_amd import sim
    s = sim.simulate(str(ring / "kernelslist.g"), "MI355X", engine="gpu")
    assert s.stats["gpgpu_n_tot_w_icount"] == sum(v for k, v in c.items() if k != "WAVES")


@pytest.mark.gpu
def test_isatrace_tiny_ring_is_lossless_or_fails(tmp_path):
    """Four 8 KB ring slots for 1024 waves: with a prompt drain the capture
    completes and equals the device-buffer capture; with the drain stalled
    (test hook) and a short poll budget, waves give up and the run fails with
    status 5 -- no kernel trace is written, the directory is marked
    CAPTURE_FAILED (never a silently truncated trace)."""
    exe = os.path.join(ROOT, "bin", "isatrace", "vectoradd")
    assert os.path.exists(exe), "build_native.py builds bin/isatrace/*"
    n = 1 << 16
    env = {k: v for k, v in os.environ.items() if not k.startswith("ASIM_TRACE")}
    ok, whole, bad = tmp_path / "ok", tmp_path / "whole", tmp_path / "bad"
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(ok), ASIM_TRACE_RING_KB="32"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(whole), ASIM_TRACE_BUF_MB="64"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert _trace_body(ok / "kernel-1.traceg") == _trace_body(whole / "kernel-1.traceg")
    assert verify.trace_counts(str(ok / "kernel-1.traceg"))["WAVES"] == n // 64
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(bad), ASIM_TRACE_RING_KB="32",
                                                ASIM_TRACE_DRAIN_DELAY_US="300000", ASIM_TRACE_SPIN_LIMIT="32"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 5, (r.returncode, r.stderr)
    assert "FATAL" in r.stderr and (bad / "CAPTURE_FAILED").exists()
    assert not [p for p in os.listdir(bad) if p.endswith(".traceg") or p.endswith(".chunks")]


@pytest.mark.gpu
def test_isatrace_ring_with_barriers_matches_device_buffer(tmp_path):
    """hotspot (workgroup barriers, several kernels) streamed through the
    default ring gives the same traces as the device-buffer mode."""
    exe = os.path.join(ROOT, "bin", "isatrace", "hotspot")
    assert os.path.exists(exe)
    env = {k: v for k, v in os.environ.items() if not k.startswith("ASIM_TRACE")}
    outs = []
    for tag, extra in (("ring", {}), ("buf", {"ASIM_TRACE_BUF_MB": "1024"})):
        d = tmp_path / tag
        r = subprocess.run([exe, "128", "2"], env=dict(env, ASIM_TRACE_DIR=str(d), **extra), capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "dropped" not in r.stderr, r.stderr
        ks = sorted(p for p in os.listdir(d) if p.endswith(".traceg"))
        outs.append({k: _trace_body(d / k) for k in ks})
    assert outs[0] and outs[0] == outs[1]


@pytest.mark.gpu
def test_isatrace_device_filter_and_rank_dirs(tmp_path):
    """GPU_TRACE_ID-style capture: only the launches on the named device are
    traced, into kernel-<id>_<gpu>.traceg; '{rank}' in ASIM_TRACE_DIR gives
    each rank of a job its own directory."""
    exe = os.path.join(ROOT, "bin", "isatrace", "vectoradd")
    env = {k: v for k, v in os.environ.items() if not k.startswith("ASIM_TRACE")}
    env.update(ASIM_TRACE_DIR=str(tmp_path / "r{rank}"), RANK="3", ASIM_TRACE_GPU_ID="0")
    r = subprocess.run([exe, "4096"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    d = tmp_path / "r3"
    assert (d / "kernel-1_0.traceg").exists() and "kernel-1_0.traceg" in (d / "kernelslist.g").read_text()
    assert verify.trace_counts(str(d / "kernel-1_0.traceg"))["WAVES"] == 4096 // 64
    # a device this process never launches on: nothing traced, the app still runs
    env.update(RANK="4", ASIM_TRACE_GPU_ID="7")
    r = subprocess.run([exe, "4096"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    assert not [p for p in os.listdir(tmp_path / "r4") if p.endswith(".traceg")]
    assert "kernel-" not in (tmp_path / "r4" / "kernelslist.g").read_text()


@pytest.mark.gpu
def test_isatrace_allocation_snapshots(tmp_path):
    """Silicon-checkpoint allocation tracking (reference checkpoint.cu:198-290):
    hipMalloc / hipFree are tracked and, with ASIM_TRACE_SNAPSHOT, every live
    allocation is written after each traced kernel; vectoradd's three buffers
    are listed and c == a + b in the snapshot."""
    import numpy as np
    exe = os.path.join(ROOT, "bin", "isatrace", "vectoradd")
    assert os.path.exists(exe), "build_native.py builds bin/isatrace/*"
    n = 4096
    env = {k: v for k, v in os.environ.items() if not k.startswith("ASIM_TRACE")}
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(tmp_path), ASIM_TRACE_SNAPSHOT="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    rows = [ln.split() for ln in (tmp_path / "kernel-1.allocs").read_text().split("\n") if ln and ln[0] != "#"]
    assert [int(x[0]) for x in rows] == [0, 1, 2] and all(int(x[2]) == n * 8 for x in rows)
    a, b, c = (np.fromfile(tmp_path / x[3], dtype=np.float64) for x in rows)
    i = np.arange(n, dtype=np.float64)
    assert np.allclose(a, np.sin(i) ** 2, atol=1e-15) and np.allclose(b, np.cos(i) ** 2, atol=1e-15)
    assert np.array_equal(c, a + b)


@pytest.mark.gpu
def test_isatrace_basic_block_vectors(tmp_path):
    """BBVs from the instrumented binary (reference bbv_count.cu): one row per
    wave, one column per basic block (rewriter segment), active threads per
    execution."""
    exe = os.path.join(ROOT, "bin", "isatrace", "vectoradd")
    n = 4096 + 100  # a partial last wave
    env = {k: v for k, v in os.environ.items() if not k.startswith("ASIM_TRACE")}
    r = subprocess.run([exe, str(n)], env=dict(env, ASIM_TRACE_DIR=str(tmp_path), ASIM_TRACE_BBV="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stderr
    lines = (tmp_path / "kernel-1.bbv").read_text().split("\n")
    assert "vecAdd" in lines[0]
    nw, nb = int(lines[1]), int(lines[2])
    rows = [[int(x) for x in ln.split()] for ln in lines[3:3 + nw]]
    assert nw == -(-n // 1024) * 16 and all(len(rw) == nb for rw in rows)
    # every wave runs the entry block with its full 64 lanes; the last wave's
    # guarded body runs with the 100 % 64 live lanes of the partial tail
    assert all(rw[0] == 64 for rw in rows)
    m = re.findall(r"vecAdd.*?, (\d+), (\d+)$", (tmp_path / "stats.csv").read_text(), re.M)
    assert m and sum(sum(rw) for rw in rows) > 0


def test_binary_path_instruments_identically():
    """A precompiled app's code object, recovered to assembly by
    isatrace/binary.py (no device source), instruments to exactly the code
    and instruction map the source path produces."""
    from accel_sim_framework_distributed_amd.isatrace import binary
    for app in ("nw", "lud", "hotspot", "backprop", "devcalls"):
        a, b = (os.path.join(ROOT, d, app) for d in ("bin/isatrace", "bin/isatrace_bin"))
        if not (os.path.exists(a) and os.path.exists(b)):
            pytest.skip("build_native.py builds bin/isatrace{,_bin}/*")
        assert open(a + ".asimisa").read() == open(b + ".asimisa").read(), app
        la = binary.disassemble(binary.extract(a, f"/tmp/asim_bin_cmp/{app}/a")[0])
        lb = binary.disassemble(binary.extract(b, f"/tmp/asim_bin_cmp/{app}/b")[0])
        assert [f.name for f in la.funcs] == [f.name for f in lb.funcs]
        assert all(binary._insn_bytes(f) == binary._insn_bytes(g) for f, g in zip(la.funcs, lb.funcs)), app
        assert la.kds == lb.kds, app


@pytest.mark.gpu
def test_binary_path_trace_equals_source_path(tmp_path):
    """On the MI355X: the binary-only traced nw captures the same trace as the
    source-built one."""
    outs = []
    for d in ("isatrace", "isatrace_bin"):
        exe = os.path.join(ROOT, "bin", d, "nw")
        assert os.path.exists(exe), "build_native.py builds bin/isatrace{,_bin}/nw"
        td = tmp_path / d
        env = dict(os.environ, ASIM_TRACE_DIR=str(td), ASIM_TRACE_BUF_MB="256")
        r = subprocess.run([exe, "128", "10"], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(td)
    ka = sorted(p.name for p in outs[0].glob("kernel-*.traceg"))
    assert ka and ka == sorted(p.name for p in outs[1].glob("kernel-*.traceg"))
    for k in ka:
        assert _trace_body(str(outs[0] / k)) == _trace_body(str(outs[1] / k)), k


def test_device_functions_are_instrumented():
    """A kernel that calls device functions: the functions get probes with the
    kernel's register window and segment ids shared by every kernel, the
    kernel's map holds the functions' segments, their PCs sit above
    FUNC_PC_BASE."""
    m = open(os.path.join(ROOT, "bin", "isatrace", "devcalls.asimisa")).read() \
        if os.path.exists(os.path.join(ROOT, "bin", "isatrace", "devcalls.asimisa")) else None
    if m is None:
        pytest.skip("build_native.py builds bin/isatrace/devcalls")
    lines = m.split("\n")
    assert sum(1 for ln in lines if ln.startswith("K ")) == 1
    pcs = [int(ln.split()[0], 16) for ln in lines if ln and ln[0] not in "KSA"]
    assert any(pc >= rewrite.FUNC_PC_BASE for pc in pcs) and any(pc < rewrite.FUNC_PC_BASE for pc in pcs)
    assert any("s_swappc_b64" in ln for ln in lines) and any("s_setpc_b64" in ln for ln in lines)


@pytest.mark.gpu
def test_device_function_trace_matches_counters(tmp_path):
    """On the MI355X: the traced devcalls computes the right answer, and the
    trace's instruction counts per SQ class (kernel + called functions) equal
    rocprofv3 SQ_INSTS_* of the plain build."""
    exe = os.path.join(ROOT, "bin", "isatrace", "devcalls")
    plain = os.path.join(ROOT, "bin", "apps", "devcalls")
    assert os.path.exists(exe) and os.path.exists(plain), "build_native.py builds bin/{apps,isatrace}/devcalls"
    td = tmp_path / "trace"
    env = dict(os.environ, ASIM_TRACE_DIR=str(td), ASIM_TRACE_BUF_MB="128")
    r = subprocess.run([exe, "4096"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout[-1000:] + r.stderr[-2000:]
    pmc = tmp_path / "pmc"
    ctr = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH",
           "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"]
    r = subprocess.run(["rocprofv3", "--pmc"] + ctr + ["--output-format", "csv", "-d", str(pmc), "-o", "run", "--",
                                                       plain, "4096"],
                       cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stderr[-2000:]
    res = verify.compare(str(td), str(pmc))
    assert res["kernels"] == 1
    for c, v in res["total"].items():
        assert v["trace"] == v["hw"], (c, v)
