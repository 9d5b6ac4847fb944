"""-network_mode 1: Booksim/intersim2 .icnt files, topology latency model
(reference gpu-simulator/gpgpu-sim/src/intersim2: networks/*, routers/
iq_router pipeline; icnt_wrapper.cc node numbering) and the pre-Volta presets
that use it."""
import glob
import re
import os
import subprocess

import pytest

from conftest import REFERENCE
from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen import rodinia

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_booksim_grammar(native):
    kv = native.parse_booksim_config("""
        // a comment
        topology = mesh; /* block
        comment */ k = 4 ;
        n=2;
        packet_size ={{1,2,3,4},{10,20}};  // list value keeps its braces
        routing_function = dim_order;""")
    assert kv["topology"] == "mesh" and kv["k"] == "4" and kv["n"] == "2"
    assert kv["packet_size"] == "{{1,2,3,4},{10,20}}"
    assert kv["routing_function"] == "dim_order"


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference tree not mounted")
def test_reference_icnt_files_parse(native):
    files = glob.glob(os.path.join(REFERENCE, "gpu-simulator/gpgpu-sim/configs/tested-cfgs/*/*.icnt"))
    assert files
    for f in files:
        kv = native.parse_booksim_config(open(f).read())
        assert kv["topology"] == "fly" and kv["n"] == "1" and int(kv["k"]) >= 27, f


def _icnt_args(tmp_path, name, **kw):
    p = tmp_path / f"{name}.icnt"
    p.write_text(presets.render_icnt(presets.icnt_params(**kw)))
    # 16 clusters + 16 sub-partitions = 32 nodes
    return presets.args_for("QV100", {"-gpgpu_n_clusters": "16", "-gpgpu_n_mem": "8",
                                      "-network_mode": "1", "-inter_config_file": str(p)})


def test_topology_latencies(native, tmp_path):
    fly = _icnt_args(tmp_path, "fly", k=32, n=1)
    lat, look, routers = native.icnt_latency(fly, 0, 0)
    assert routers == 1 and look == int(lat) and lat == 5  # 1 router x (0+1+1+1) + 2 channels
    mesh = _icnt_args(tmp_path, "mesh", k=8, n=2, topology="mesh")
    # node 0 (SM 0) -> node 16 + 15 = 31: (7, 3) in an 8x8 mesh: 7 + 3 hops, 11 routers
    assert native.icnt_latency(mesh, 0, 15)[2] == 11
    torus = _icnt_args(tmp_path, "torus", k=8, n=2, topology="torus")
    assert native.icnt_latency(torus, 0, 15)[2] == 1 + 1 + 3  # wrap-around in x
    ft = _icnt_args(tmp_path, "ft", k=4, n=3, topology="fattree")
    assert native.icnt_latency(ft, 0, 0)[2] == 5   # leaves 0 and 16 share only the root level
    # lookahead = the smallest pair latency in core cycles
    assert native.icnt_latency(mesh, 0, 0)[1] <= min(native.icnt_latency(mesh, s, d)[0]
                                                    for s in range(16) for d in range(16))


def test_too_small_topology_rejected(native, tmp_path):
    small = _icnt_args(tmp_path, "small", k=8, n=1)
    with pytest.raises(Exception):
        native.parse_config(small)


def test_mesh_slower_than_crossbar(native, tmp_path):
    kl = rodinia.write_app(str(tmp_path / "bfs"), rodinia.bfs(2048, levels=2))
    runs = {}
    for name, kw in (("fly", dict(k=32, n=1)), ("mesh", dict(k=8, n=2, topology="mesh"))):
        s = native.Simulator(_icnt_args(tmp_path, name, **kw) + ["-trace", kl], False)
        assert s.run() == 0 and not s.deadlock
        runs[name] = s
    assert runs["fly"].tot_insn == runs["mesh"].tot_insn
    assert runs["mesh"].tot_cycle > runs["fly"].tot_cycle


@pytest.mark.parametrize("preset", ["GTX480", "KEPLER_TITAN", "TITANX", "RTX2060_S"])
def test_pre_volta_presets(native, tmp_path, preset):
    kl = rodinia.write_app(str(tmp_path / "vadd"), [rodinia.vectoradd(20000, block=256)])
    s = native.Simulator(presets.args_for(preset) + ["-trace", kl], False)
    q = native.Simulator(presets.args_for("QV100") + ["-trace", kl], False)
    assert s.run() == 0 and q.run() == 0
    assert s.tot_insn == q.tot_insn and s.tot_cycle > 0 and not s.deadlock
    # written run directories carry the interconnect file and run from anywhere
    d = tmp_path / "cfg"
    presets.write_config(preset, str(d))
    args = [os.path.join(ROOT, "bin", "accel-sim.out"), "-config", str(d / "gpgpusim.config"),
            "-config", str(d / "trace.config"), "-trace", kl]
    p = subprocess.run(args, cwd="/", capture_output=True, text=True)
    assert p.returncode == 0, p.stdout[-500:] + p.stderr[-500:]
    assert "gpu_tot_sim_cycle" in p.stdout


def test_epoch_length_sensitivity_is_smooth(tmp_path):
    """-icnt_latency is both the crossbar latency and the PDES lookahead: short
    epochs must still simulate (multi-flit packets serialise across epoch
    boundaries) and cycles must grow smoothly with the latency, not jump."""
    from accel_sim_framework_distributed_amd import sim
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    kls = rodinia.generate_suite(str(tmp_path), ["nn-rodinia-2.0-ft", "backprop-rodinia-2.0-ft"])
    for app, kl in kls.items():
        cyc = []
        for L in (1, 2, 8):
            r = sim.simulate(kl, "GV100", engine="cpu", extra={"-icnt_latency": str(L)})
            assert not r.deadlock, (app, L)
            cyc.append(r.tot_cycle)
        assert cyc[0] <= cyc[1] * 1.01 and cyc[1] <= cyc[2] * 1.01, (app, cyc)
        assert cyc[2] <= cyc[0] * 1.10, (app, cyc)  # 7 extra cycles per hop cost < 10 %


# ---- crossbar output-port arbitration (local_interconnect.cc:123-270) -------
def _hotspot_app(tmp_path, name, same_line):
    """80 single-warp CTAs; each warp issues 16 independent loads.  same_line:
    every SM reads the same lines, whose requests all meet at ONE L2
    sub-partition's port (a hotspot); else each SM reads its own lines,
    spread over all sub-partitions."""
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    import numpy as np
    k = KernelBuilder("_Z7hotspotPf", (80, 1, 1), (32, 1, 1), nregs=32)
    g = k.g
    for i in range(16):
        if same_line:
            base = np.full(g.nwarps, 0x7000_0000 + i * 0x40000, np.int64)
            k.op("LDG.E", [8 + i], [2], base=base, stride=0)
        else:
            k.op("LDG.E", [8 + i], [2], base=0x7000_0000 + g.cta * 0x100000 + i * 128, stride=4)
    for i in range(16):
        k.op("FADD", [5], [8 + i, 5])
    k.op("EXIT")
    return rodinia.write_app(str(tmp_path / name), [k.build()], memcpy=False)


def _stat(out, key):
    import re
    m = re.findall(rf"^{re.escape(key)} = ([0-9.]+)", out, re.M)
    return float(m[-1])


@pytest.mark.parametrize("algo", ["0", "1"])
def test_crossbar_hotspot_queues_at_one_port(native, tmp_path, algo):
    outs = {}
    for hot in (True, False):
        kl = _hotspot_app(tmp_path, f"h{int(hot)}_{algo}", hot)
        s = native.Simulator(presets.args_for("QV100", {"-icnt_arbiter_algo": algo, "-gpgpu_perf_sim_memcpy": "0"})
                             + ["-trace", kl], False)
        assert s.run() == 0
        outs[hot] = s.output
    hot, spread = outs[True], outs[False]
    # every SM's miss for the same line meets at one port: conflicts and queueing
    assert _stat(hot, "Req_Network_conflicts") > 100
    assert _stat(hot, "Req_Network_avg_queueing_cycles") > 5 * max(0.5, _stat(spread, "Req_Network_avg_queueing_cycles"))
    assert _stat(hot, "Req_Network_injected_packets_num") == _stat(spread, "Req_Network_injected_packets_num") == 80 * 16


@pytest.mark.gpu
def test_crossbar_hotspot_gpu_matches_cpu(native, tmp_path):
    kl = _hotspot_app(tmp_path, "hg", True)
    res = []
    for eng in ("cpu", "gpu"):
        s = native.Simulator(presets.args_for("QV100", {"-gpgpu_perf_sim_memcpy": "0", "-sim_engine": eng})
                             + ["-trace", kl], False)
        assert s.run() == 0
        res.append([_stat(s.output, k) for k in ("gpu_sim_cycle", "Req_Network_conflicts",
                                                  "Req_Network_queueing_cycles", "Reply_Network_queueing_cycles")])
    assert res[0] == res[1] and res[0][1] > 100


# ---- link-level contention in multi-hop topologies (icnt_links.h) ----------
TOPOS = [("mesh", dict(k=8, n=2, topology="mesh")), ("torus", dict(k=8, n=2, topology="torus")),
         ("fly2", dict(k=8, n=2, topology="fly")), ("fattree", dict(k=4, n=3, topology="fattree")),
         ("flatfly", dict(k=8, n=2, topology="flatfly")),
         # concentrated flatfly_onchip: k^n = 16 routers < 32 endpoints, 2 terminals per router
         ("flatfly_conc", dict(k=4, n=2, c=2, topology="flatfly"))]


@pytest.mark.parametrize("name,kw", TOPOS)
def test_link_routes_follow_the_topology(native, tmp_path, name, kw):
    args = _icnt_args(tmp_path, name, **kw)
    for a in range(16):
        for sub in range(16):
            b = 16 + sub
            for (x, y) in ((a, b), (b, a)):
                links, total = native.icnt_path(args, x, y)
                # one link per router crossed (the last one ejects), as many as
                # the latency model's router count, all distinct and in range
                sm = x if x < 16 else y
                assert len(links) == native.icnt_latency(args, sm, sub)[2], (name, x, y)
                assert len(set(links)) == len(links) and all(0 <= l < total for l in links)
            # routes to different destinations leave through different ejection links
    ej = {native.icnt_path(args, 0, 16 + s)[0][-1] for s in range(16)}
    assert len(ej) == 16


def test_flatfly_with_fewer_nodes_than_endpoints_is_rejected(native, tmp_path):
    # k^n = 16 routers without concentration cannot hold 32 endpoints: the link
    # pass would index past its table, so the config is refused
    args = _icnt_args(tmp_path, "ff_small", k=4, n=2, topology="flatfly")
    with pytest.raises(Exception, match="nodes"):
        native.Simulator(args + ["-icnt_link_contention", "1", "-trace", "/nonexistent"], False)


def test_concentrated_flatfly_contention_runs(native, tmp_path):
    kl = _hotspot_app(tmp_path, "ffc", True)
    args = _icnt_args(tmp_path, "ffc", k=4, n=2, c=2, topology="flatfly")
    s = native.Simulator(args + ["-icnt_link_contention", "1", "-gpgpu_perf_sim_memcpy", "0", "-trace", kl], False)
    assert s.run() == 0 and not s.deadlock
    assert _link_stat(s.output, "Network_link_delayed_packets") > 0


def test_single_stage_crossbar_has_no_internal_links(native, tmp_path):
    fly = _icnt_args(tmp_path, "fly", k=32, n=1)
    assert native.icnt_path(fly, 0, 16) == ([], 0)
    kl = rodinia.write_app(str(tmp_path / "bfs"), rodinia.bfs(2048, levels=2))
    res = []
    for lc in ("0", "1"):
        s = native.Simulator(fly + ["-icnt_link_contention", lc, "-trace", kl], False)
        assert s.run() == 0
        res.append((s.tot_cycle, s.output.count("Network_link_wait_cycles")))
    assert res[0] == (res[1][0], 0) and res[1][1] == 0  # identical, nothing to report


def _link_stat(out, key):
    return int(re.findall(rf"^{key} = (\d+)", out, re.M)[-1])


def test_mesh_hotspot_links_delay_packets(native, tmp_path):
    kl = _hotspot_app(tmp_path, "hot", True)
    mesh = _icnt_args(tmp_path, "mesh", k=8, n=2, topology="mesh")
    runs = {}
    for lc in ("0", "1"):
        s = native.Simulator(mesh + ["-icnt_link_contention", lc, "-gpgpu_perf_sim_memcpy", "0", "-trace", kl], False)
        assert s.run() == 0 and not s.deadlock
        runs[lc] = s
    assert runs["0"].tot_insn == runs["1"].tot_insn
    assert "Network_link_wait_cycles" not in runs["0"].output
    out = runs["1"].output
    assert _link_stat(out, "Network_link_delayed_packets") > 100
    assert _link_stat(out, "Network_link_wait_cycles") > _link_stat(out, "Network_link_delayed_packets")
    # 80 SMs' requests converge on one sub-partition: shared links cost time
    assert runs["1"].tot_cycle > runs["0"].tot_cycle
    # deterministic, and independent of the CPU engine's thread count
    s4 = native.Simulator(mesh + ["-icnt_link_contention", "1", "-gpgpu_perf_sim_memcpy", "0",
                                  "-sim_cpu_threads", "4", "-trace", kl], False)
    assert s4.run() == 0
    assert (s4.tot_cycle, _link_stat(s4.output, "Network_link_wait_cycles")) == \
        (runs["1"].tot_cycle, _link_stat(out, "Network_link_wait_cycles"))


def test_link_state_checkpoint_resumes_exactly(native, tmp_path):
    from accel_sim_framework_distributed_amd.tracegen import rodinia as rd
    kl = rd.write_app(str(tmp_path / "pf"), rd.pathfinder(4000, 12, 2))
    mesh = _icnt_args(tmp_path, "mesh", k=8, n=2, topology="mesh") + [
        "-icnt_link_contention", "1", "-trace", kl, "-checkpoint_path", str(tmp_path / "ck")]
    full = native.Simulator(mesh, False)
    assert full.run() == 0
    first = native.Simulator(mesh + ["-checkpoint_option", "1", "-checkpoint_kernel", "2"], False)
    assert first.run() == 0
    rest = native.Simulator(mesh + ["-resume_option", "1", "-resume_kernel", "2"], False)
    assert rest.run() == 0 and "resumed from" in rest.output
    assert rest.tot_cycle == full.tot_cycle and _link_stat(full.output, "Network_link_delayed_packets") > 0
    assert _link_stat(rest.output, "Network_link_wait_cycles") == _link_stat(full.output, "Network_link_wait_cycles")


@pytest.mark.gpu
def test_mesh_link_contention_gpu_matches_cpu(native, tmp_path):
    kl = _hotspot_app(tmp_path, "hotg", True)
    mesh = _icnt_args(tmp_path, "mesh", k=8, n=2, topology="mesh")
    res = []
    for eng in ("cpu", "gpu"):
        s = native.Simulator(mesh + ["-icnt_link_contention", "1", "-gpgpu_perf_sim_memcpy", "0",
                                     "-sim_engine", eng, "-trace", kl], False)
        assert s.run() == 0
        res.append((s.tot_cycle, _link_stat(s.output, "Network_link_delayed_packets"),
                    _link_stat(s.output, "Network_link_wait_cycles"), _stat(s.output, "Req_Network_queueing_cycles")))
    assert res[0] == res[1] and res[0][1] > 100


# ---- input-queued router microarchitecture (icnt_router.h) -----------------
def _rt_icnt(**kw):
    base = dict(vc_buf_size="8", internal_speedup="1.0")
    base.update(kw)
    return presets.render_icnt(presets.icnt_params(**base))


def test_router_crossbar_head_of_line_blocking(native):
    """A FIFO input-queued crossbar under uniform traffic saturates near
    2 - sqrt(2) = 58.6 % (head-of-line blocking); an internal speedup of 2
    lifts it well above; below saturation latency is the zero-load latency."""
    xbar = _rt_icnt(k=32, n=1)
    sat = native.icnt_open_loop(xbar, "uniform", 1.0, 1, 3000, 1000, 1)
    assert 0.56 < sat["accepted"] < 0.63 and sat["deadlocked"] == 0
    fast = native.icnt_open_loop(_rt_icnt(k=32, n=1, internal_speedup="2.0"), "uniform", 1.0, 1, 3000, 1000, 1)
    assert fast["accepted"] > 0.85
    low = native.icnt_open_loop(xbar, "uniform", 0.1, 1, 3000, 1000, 1)
    assert abs(low["accepted"] - 0.1) < 0.01
    assert low["zero_load_latency"] == 5 and low["avg_latency"] < 5.3
    # the allocators differ in pointer policy only; all are work conserving here
    sep = native.icnt_open_loop(_rt_icnt(k=32, n=1, sw_allocator="separable_input_first"), "uniform", 1.0, 1,
                                3000, 1000, 1)
    assert 0.56 < sep["accepted"] < 0.63
    # virtual channels at the inputs relieve head-of-line blocking
    vcs = native.icnt_open_loop(_rt_icnt(k=32, n=1, num_vcs="4"), "uniform", 1.0, 1, 3000, 1000, 1)
    assert vcs["accepted"] >= sat["accepted"]


def test_router_mesh_saturates_below_bisection(native):
    mesh = _rt_icnt(k=8, n=2, topology="mesh")
    sat = native.icnt_open_loop(mesh, "uniform", 1.0, 1, 3000, 1000, 1)
    # bisection bound of an 8x8 mesh under uniform traffic: 4 / k = 0.5
    assert 0.3 < sat["accepted"] < 0.5 and sat["deadlocked"] == 0
    low = native.icnt_open_loop(mesh, "uniform", 0.1, 1, 3000, 1000, 1)
    assert low["avg_latency"] < 1.05 * low["zero_load_latency"]
    # transpose concentrates dimension-order routes on the diagonal's links
    tr = native.icnt_open_loop(mesh, "transpose", 1.0, 1, 3000, 1000, 1)
    assert tr["accepted"] < sat["accepted"]
    # multi-flit packets: serialisation is part of the zero-load latency
    four = native.icnt_open_loop(mesh, "uniform", 0.05, 4, 3000, 1000, 1)
    assert abs(four["zero_load_latency"] - low["zero_load_latency"] - 3) < 0.5
    assert four["avg_latency"] < 1.1 * four["zero_load_latency"]


def test_router_torus_dateline_classes(native):
    """Dimension-order routing on a torus needs two VC classes (dateline):
    with one VC the ring deadlocks under load and the pass reports it."""
    one = native.icnt_open_loop(_rt_icnt(k=8, n=2, topology="torus"), "uniform", 1.0, 1, 2000, 500, 1)
    assert one["deadlocked"] > 0
    two = native.icnt_open_loop(_rt_icnt(k=8, n=2, topology="torus", num_vcs="2"), "uniform", 1.0, 1, 2000, 500, 1)
    assert two["deadlocked"] == 0 and two["accepted"] > 0.35


def test_router_traffic_patterns_are_deterministic(native):
    mesh = _rt_icnt(k=4, n=2, topology="mesh")
    for t in ("uniform", "transpose", "bitcomp", "bitrev", "shuffle", "tornado", "neighbor"):
        a = native.icnt_open_loop(mesh, t, 0.3, 2, 1000, 200, 7)
        b = native.icnt_open_loop(mesh, t, 0.3, 2, 1000, 200, 7)
        assert a == b and a["packets"] > 0, t
    with pytest.raises(Exception, match="traffic"):
        native.icnt_open_loop(mesh, "nonesuch", 0.3, 1, 1000, 200, 1)


def test_router_model_in_the_simulator(native, tmp_path):
    kl = _hotspot_app(tmp_path, "rt", True)
    mesh = _icnt_args(tmp_path, "rtmesh", k=8, n=2, topology="mesh")
    runs = {}
    for lc in ("0", "2"):
        s = native.Simulator(mesh + ["-icnt_link_contention", lc, "-gpgpu_perf_sim_memcpy", "0", "-trace", kl], False)
        assert s.run() == 0 and not s.deadlock
        runs[lc] = s
    assert runs["0"].tot_insn == runs["2"].tot_insn
    out = runs["2"].output
    assert _link_stat(out, "Network_link_delayed_packets") > 50
    assert runs["2"].tot_cycle >= runs["0"].tot_cycle
    s4 = native.Simulator(mesh + ["-icnt_link_contention", "2", "-gpgpu_perf_sim_memcpy", "0",
                                  "-sim_cpu_threads", "4", "-trace", kl], False)
    assert s4.run() == 0
    assert (s4.tot_cycle, _link_stat(s4.output, "Network_link_wait_cycles")) == \
        (runs["2"].tot_cycle, _link_stat(out, "Network_link_wait_cycles"))
    # the single-stage crossbar's output ports are arbitrated too
    fly = _icnt_args(tmp_path, "rtfly", k=32, n=1)
    s = native.Simulator(fly + ["-icnt_link_contention", "2", "-gpgpu_perf_sim_memcpy", "0", "-trace", kl], False)
    assert s.run() == 0 and _link_stat(s.output, "Network_link_delayed_packets") > 0
    assert native.icnt_path(fly + ["-icnt_link_contention", "2"], 0, 16) == ([16], 32)


def test_router_state_checkpoint_resumes_exactly(native, tmp_path):
    from accel_sim_framework_distributed_amd.tracegen import rodinia as rd
    kl = rd.write_app(str(tmp_path / "pf"), rd.pathfinder(4000, 12, 2))
    mesh = _icnt_args(tmp_path, "mesh", k=8, n=2, topology="mesh") + [
        "-icnt_link_contention", "2", "-trace", kl, "-checkpoint_path", str(tmp_path / "ck")]
    full = native.Simulator(mesh, False)
    assert full.run() == 0
    first = native.Simulator(mesh + ["-checkpoint_option", "1", "-checkpoint_kernel", "2"], False)
    assert first.run() == 0
    rest = native.Simulator(mesh + ["-resume_option", "1", "-resume_kernel", "2"], False)
    assert rest.run() == 0 and "resumed from" in rest.output
    assert rest.tot_cycle == full.tot_cycle
    assert _link_stat(rest.output, "Network_link_wait_cycles") == _link_stat(full.output, "Network_link_wait_cycles")


def test_router_unmodelled_allocator_refused_only_when_used(native, tmp_path):
    p = tmp_path / "wf.icnt"
    p.write_text(presets.render_icnt(presets.icnt_params(k=32, sw_allocator="select")))
    args = presets.args_for("QV100", {"-gpgpu_n_clusters": "16", "-gpgpu_n_mem": "8",
                                      "-network_mode": "1", "-inter_config_file": str(p)})
    native.parse_config(args)  # the latency model does not need the allocator
    with pytest.raises(Exception, match="sw_allocator"):
        native.parse_config(args + ["-icnt_link_contention", "2"])
    with pytest.raises(Exception, match="icnt_link_contention"):
        native.parse_config(args + ["-icnt_link_contention", "3"])


@pytest.mark.gpu
def test_router_model_gpu_matches_cpu(native, tmp_path):
    kl = _hotspot_app(tmp_path, "rtg", True)
    for name, kw in (("mesh", dict(k=8, n=2, topology="mesh")), ("fly", dict(k=32, n=1)),
                     ("mesh_adapt", dict(k=8, n=2, topology="mesh", num_vcs="4", routing_function="min_adapt")),
                     ("fly_maxsize", dict(k=32, n=1, num_vcs="2", sw_allocator="max_size")),
                     ("mesh_valiant", dict(k=8, n=2, topology="mesh", num_vcs="2", routing_function="valiant"))):
        args = _icnt_args(tmp_path, name, **kw)
        res = []
        for eng in ("cpu", "gpu"):
            s = native.Simulator(args + ["-icnt_link_contention", "2", "-gpgpu_perf_sim_memcpy", "0",
                                         "-sim_engine", eng, "-trace", kl], False)
            assert s.run() == 0
            res.append((s.tot_cycle, _link_stat(s.output, "Network_link_delayed_packets"),
                        _link_stat(s.output, "Network_link_wait_cycles")))
        assert res[0] == res[1] and res[0][1] > 0, name


def test_router_allocators_match_quality(native):
    """With 4 VCs per input a crossbar input offers several outputs, so the
    switch allocator's matching quality shows: a maximum-size matching beats
    the wavefront allocator, which beats one iteration of iSLIP; more iSLIP
    iterations help; every allocator is deterministic and deadlock free."""
    sat = {}
    for al in ("islip", "separable_input_first", "separable_output_first", "wavefront", "max_size", "pim", "loa"):
        t = _rt_icnt(k=32, n=1, num_vcs="4", sw_allocator=al)
        r = native.icnt_open_loop(t, "uniform", 1.0, 1, 2000, 500, 3)
        assert r == native.icnt_open_loop(t, "uniform", 1.0, 1, 2000, 500, 3) and r["deadlocked"] == 0, al
        sat[al] = r["accepted"]
        low = native.icnt_open_loop(t, "uniform", 0.1, 1, 2000, 500, 3)
        assert low["avg_latency"] < 1.1 * low["zero_load_latency"], al
    assert sat["max_size"] >= sat["wavefront"] > sat["islip"] + 0.1
    it4 = native.icnt_open_loop(_rt_icnt(k=32, n=1, num_vcs="4", alloc_iters="4"), "uniform", 1.0, 1, 2000, 500, 3)
    assert it4["accepted"] > sat["islip"] + 0.05


def test_router_minimal_adaptive_routing(native):
    """min_adapt on a mesh (Duato: VC 0 the dimension-order escape channel,
    the other VCs adaptive over the productive directions): transpose traffic,
    which piles dimension-order routes onto few links, drains much faster;
    no deadlock, deterministic, the zero-load latency unchanged."""
    kw = dict(k=8, n=2, topology="mesh", num_vcs="4")
    dor = _rt_icnt(**kw)
    ada = _rt_icnt(routing_function="min_adapt", **kw)
    a = native.icnt_open_loop(ada, "transpose", 1.0, 1, 2000, 500, 1)
    d = native.icnt_open_loop(dor, "transpose", 1.0, 1, 2000, 500, 1)
    # saturated open loop: the rate the bottleneck drains every queued packet at
    assert a["deadlocked"] == 0 and a["drain_throughput"] > 1.3 * d["drain_throughput"]
    assert a == native.icnt_open_loop(ada, "transpose", 1.0, 1, 2000, 500, 1)
    lo_a = native.icnt_open_loop(ada, "uniform", 0.05, 1, 2000, 500, 1)
    lo_d = native.icnt_open_loop(dor, "uniform", 0.05, 1, 2000, 500, 1)
    assert lo_a["zero_load_latency"] == lo_d["zero_load_latency"]
    assert lo_a["avg_latency"] < 1.05 * lo_a["zero_load_latency"]
    u = native.icnt_open_loop(ada, "uniform", 1.0, 2, 2000, 500, 1)
    assert u["deadlocked"] == 0 and u["accepted"] > 0.3


def test_booksim_standalone_cli(tmp_path, capsys):
    """python -m accel_sim_framework_distributed_amd.icnt.booksim: Booksim's
    standalone mode over a .icnt file, one block per injection rate and a JSON
    curve."""
    from accel_sim_framework_distributed_amd.icnt import booksim
    f = tmp_path / "x.icnt"
    f.write_text(_rt_icnt(k=16, n=1))
    out = tmp_path / "curve.json"
    assert booksim.main([str(f), "--rates", "0.1,1.0", "--cycles", "1500", "--warmup", "300",
                         "--json", str(out)]) == 0
    text = capsys.readouterr().out
    assert text.count("Overall average latency") == 2 and "Saturation" in text
    import json
    curve = json.load(open(out))["curve"]
    assert [c["rate"] for c in curve] == [0.1, 1.0]
    assert curve[1]["accepted"] < 0.75 and booksim.saturation(curve) == 0.1


def test_router_activity_and_network_power(native):
    """Booksim's power-module inputs: every delivered flit is written into and
    read out of one input buffer per router it crosses plus the injection
    buffer, crosses one link per hop (the last an ejection link); energy grows
    with load and each per-event energy key scales its component."""
    mesh = _rt_icnt(k=4, n=2, topology="mesh")
    r = native.icnt_open_loop(mesh, "uniform", 0.2, 2, 1500, 300, 5)
    a = r["activity"]
    flits = 2 * r["packets"]
    assert a["eject_flits"] == flits
    assert a["buffer_writes"] == a["buffer_reads"] == a["link_flits"] + a["eject_flits"]
    # (the credits of the last flits are still in flight when the pass ends)
    assert 0 <= a["buffer_reads"] - a["credits"] < 64 and a["sa_requests"] >= a["buffer_reads"]
    hi = native.icnt_open_loop(mesh, "uniform", 0.4, 2, 1500, 300, 5)
    assert hi["power_w"] > r["power_w"] > 0
    twice = native.icnt_open_loop(_rt_icnt(k=4, n=2, topology="mesh", power_link_pj_per_bit_mm="0.3"),
                                  "uniform", 0.2, 2, 1500, 300, 5)
    assert abs(twice["energy_pj"]["link"] - 2 * r["energy_pj"]["link"]) < 1e-6 * r["energy_pj"]["link"]
    assert twice["energy_pj"]["buffer"] == r["energy_pj"]["buffer"]


def test_router_anynet_network_file(native, tmp_path):
    """Booksim anynet: an explicit router / node graph with per-channel
    latencies, routed along the fewest-delay paths.  A 4x4 mesh written as an
    anynet file has the built-in mesh's zero-load latency; a slow channel
    shows up in the latency of the packets that cross it."""
    k = 4
    lines = []
    for y in range(k):
        for x in range(k):
            r = y * k + x
            parts = [f"router {r}", f"node {r}"]
            if x + 1 < k:
                parts.append(f"router {r + 1}")
            if y + 1 < k:
                parts.append(f"router {r + k}")
            lines.append(" ".join(parts))
    f = tmp_path / "mesh44.anynet"
    f.write_text("\n".join(lines) + "\n")
    any_t = _rt_icnt(k=4, topology="anynet", network_file=str(f))
    mesh_t = _rt_icnt(k=4, n=2, topology="mesh")
    a = native.icnt_open_loop(any_t, "uniform", 0.1, 1, 2000, 500, 1)
    m = native.icnt_open_loop(mesh_t, "uniform", 0.1, 1, 2000, 500, 1)
    assert a["zero_load_latency"] == m["zero_load_latency"] and a["deadlocked"] == 0
    assert abs(a["avg_latency"] - m["avg_latency"]) < 0.5
    assert a == native.icnt_open_loop(any_t, "uniform", 0.1, 1, 2000, 500, 1)
    # two routers joined by a 5-cycle channel (1 cycle back), one node each
    g = tmp_path / "pair.anynet"
    g.write_text("router 0 node 0 router 1 5\nrouter 1 node 1\n")
    p = native.icnt_open_loop(_rt_icnt(k=2, topology="anynet", network_file=str(g)), "uniform", 0.01, 1, 4000, 500, 1)
    # injection 1 + (router 3 + channel) per router: 0 -> 1 crosses the 5-cycle
    # channel, 1 -> 0 the 1-cycle one; ejection channels 1 cycle
    assert p["zero_load_latency"] == pytest.approx(1 + 3 + 3 + 1 + (5 + 1) / 2, abs=0.6)


def test_router_valiant_routing(native):
    """Valiant (mesh, 2 VC classes): dimension order to a random intermediate
    router, then to the destination -- about half the uniform-traffic
    throughput of dimension order and about twice its low-load latency; no
    deadlock; reproducible."""
    kw = dict(k=8, n=2, topology="mesh", num_vcs="4")
    dor = _rt_icnt(**kw)
    val = _rt_icnt(routing_function="valiant", **kw)
    d = native.icnt_open_loop(dor, "uniform", 1.0, 1, 2000, 500, 1)
    v = native.icnt_open_loop(val, "uniform", 1.0, 1, 2000, 500, 1)
    assert v["deadlocked"] == 0 and 0.3 < v["drain_throughput"] / d["drain_throughput"] < 0.7
    lo = native.icnt_open_loop(val, "uniform", 0.05, 1, 2000, 500, 1)
    assert lo["avg_latency"] > 1.5 * lo["zero_load_latency"]
    assert lo == native.icnt_open_loop(val, "uniform", 0.05, 1, 2000, 500, 1)


def _store_app(tmp_path, name, stores):
    """80 single-warp CTAs, each storing `stores` full lines (5-flit write
    packets) to the same L2 sub-partition: offered load grows with `stores`."""
    from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder
    import numpy as np
    k = KernelBuilder("_Z6storesPf", (80, 1, 1), (32, 1, 1), nregs=32)
    for i in range(stores):
        base = 0x7000_0000 + np.arange(k.g.nwarps, dtype=np.int64) * 0x100000 + i * 0x40000
        k.op("STG.E", [], [2, 3], base=base, stride=4)
    k.op("EXIT")
    return rodinia.write_app(str(tmp_path / name), [k.build()], memcpy=False)


def test_router_back_pressure_throttles_injection(native, tmp_path):
    """-icnt_link_contention 2: a node's injection queue holds
    input_buffer_size flits (InterconnectInterface::HasBuffer); a full queue
    stalls the SM's injection, so its stall cycles rise with the offered load,
    and a roomier queue stalls less.  Deterministic with CPU threads."""
    def run(stores, inbuf, threads=1):
        icnt = _icnt_args(tmp_path, f"bp{inbuf}", k=8, n=2, topology="mesh", input_buffer_size=inbuf,
                          vc_buf_size=4, internal_speedup="1.0")
        s = native.Simulator(icnt + ["-icnt_link_contention", "2", "-gpgpu_perf_sim_memcpy", "0",
                                     "-sim_cpu_threads", str(threads), "-trace",
                                     _store_app(tmp_path, f"st{stores}", stores)], False)
        assert s.run() == 0 and not s.deadlock
        return (_link_stat(s.output, "Req_Network_injection_stall_cycles"),
                _link_stat(s.output, "Req_Network_injected_packets_num"), s.tot_cycle,
                _link_stat(s.output, "Network_router_deadlocked_packets"))
    light, heavy = run(4, 9), run(32, 9)
    assert heavy[0] > 0 and heavy[3] == 0
    assert heavy[0] / heavy[1] > light[0] / max(1, light[1])  # stall per packet rises with load
    roomy = run(32, 4096)
    assert roomy[0] < heavy[0] and roomy[1] == heavy[1]
    assert run(32, 9, threads=4) == heavy


def test_router_model_refuses_deadlock_prone_configs(native, tmp_path):
    for name, kw in (("torus1", dict(k=8, n=2, topology="torus")),
                     ("adapt1", dict(k=8, n=2, topology="mesh", routing_function="min_adapt")),
                     ("valiant1", dict(k=8, n=2, topology="mesh", routing_function="valiant"))):
        args = _icnt_args(tmp_path, name, **kw)
        native.parse_config(args + ["-icnt_link_contention", "1"])
        with pytest.raises(Exception, match="num_vcs"):
            native.parse_config(args + ["-icnt_link_contention", "2"])
    ok = _icnt_args(tmp_path, "torus2", k=8, n=2, topology="torus", num_vcs="2")
    native.parse_config(ok + ["-icnt_link_contention", "2"])


@pytest.mark.gpu
def test_router_back_pressure_gpu_matches_cpu(native, tmp_path):
    icnt = _icnt_args(tmp_path, "bpg", k=8, n=2, topology="mesh", input_buffer_size=9, vc_buf_size=4,
                      internal_speedup="1.0")
    kl = _store_app(tmp_path, "stg", 32)
    res = []
    for eng in ("cpu", "gpu"):
        s = native.Simulator(icnt + ["-icnt_link_contention", "2", "-gpgpu_perf_sim_memcpy", "0",
                                     "-sim_engine", eng, "-trace", kl], False)
        assert s.run() == 0
        res.append((s.tot_cycle, _link_stat(s.output, "Req_Network_injection_stall_cycles"),
                    _link_stat(s.output, "Reply_Network_injection_stall_cycles"),
                    _link_stat(s.output, "Network_link_wait_cycles")))
    assert res[0] == res[1] and res[0][1] > 0
