"""Multi-rank simulation over torch.distributed (gloo on CPU, world size 2).

Checks that the RCCL/xGMI epoch protocol of the packet-level link model
(parallel/collectives.py) reproduces the single-process emulation exactly,
that arrival skew between ranks is honoured, and that the all-reduce example
(examples/all-reduce of the reference) runs one simulated GPU per rank.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

from accel_sim_framework_distributed_amd.parallel import collectives

PARAMS = dict(link_gbps=153.0, latency_ns=1000.0, links=7, slice_bytes=65536, max_channels=16, reduce_gbps=900.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    import torch.distributed as dist
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ex = collectives.PacketExchange()
        out = []
        for kind, nbytes, starts in cases:
            r = ex.run(PARAMS, kind, nbytes, 0, starts[rank])
            out.append(r["finish_ps"])
        q.put((rank, out, ex.stats))
    finally:
        dist.destroy_process_group()


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda x: x[0])


def test_linksim_local_properties(native):
    S = 32 << 20
    one = collectives.emulate(PARAMS, "AllReduce", S, [0, 0])
    # 2 ranks, one link: ring all-reduce moves 2(N-1)/N * S over it
    ideal_ps = S / 153.0 * 1000
    t = max(one["finish_ps"])
    assert ideal_ps < t < ideal_ps * 1.05 + 3e6
    # more ranks -> more disjoint rings -> faster
    t8 = max(collectives.emulate(PARAMS, "AllReduce", S, [0] * 8)["finish_ps"])
    assert t8 < t
    # a late rank delays everybody's completion by about the skew
    late = collectives.emulate(PARAMS, "AllReduce", S, [0, 50_000_000])
    assert max(late["finish_ps"]) >= t + 50_000_000 - 1_000_000
    # all-to-all is cheaper than all-reduce; broadcast with one rank is free
    assert max(collectives.emulate(PARAMS, "AllToAll", S, [0] * 4)["finish_ps"]) < \
        max(collectives.emulate(PARAMS, "AllReduce", S, [0] * 4)["finish_ps"])
    assert collectives.emulate(PARAMS, "Broadcast", S, [7])["finish_ps"] == [7]


@pytest.mark.slow
def test_packet_exchange_matches_local_emulation(native):
    cases = [("AllReduce", 8 << 20, [0, 0]), ("AllReduce", 8 << 20, [3_000_000, 0]),
             ("AllGather", 4 << 20, [0, 1_000_000]), ("Reduce", 2 << 20, [0, 0]), ("AllToAll", 4 << 20, [5, 9])]
    res = _spawn(_worker, 2, cases)
    for i, (kind, nbytes, starts) in enumerate(cases):
        ref = collectives.emulate(PARAMS, kind, nbytes, starts)["finish_ps"]
        got = [res[r][1][i] for r in range(2)]
        assert got == ref, (kind, got, ref)
    assert res[0][2]["epochs"] > 0 and res[0][2]["packets"] > 0


def _suite_worker(rank, world, port, tdir, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from accel_sim_framework_distributed_amd.parallel.multi_gpu import DistributedSuite
        s = DistributedSuite(tdir, config="QV100", engine="cpu", rank=rank, world=world, apps=["vectoradd"])
        r = s.step()
        q.put((rank, r, s.sync.events))
    finally:
        dist.destroy_process_group()


def test_distributed_allreduce_example(native, tmp_path):
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    tdir = str(tmp_path)
    rodinia.write_app(os.path.join(tdir, "vectoradd", "NO_ARGS", "traces"), [rodinia.vectoradd(4096)])
    rodinia.write_allreduce_example(os.path.join(tdir, "all-reduce"), nranks=2, count=1 << 20)
    res = _spawn(_suite_worker, 2, tdir)
    ev0, ev1 = res[0][2], res[1][2]
    assert len(ev0) == len(ev1) == 1 and ev0[0]["mode"] == "rccl"
    assert ev0[0]["cycles"] == ev1[0]["cycles"] > 0
    # matches the standalone simulator's local emulation of both ranks
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.sim import build_args
    sim = _native.load().Simulator(build_args("QV100", os.path.join(tdir, "all-reduce", "kernelslist.g"), "cpu",
                                              {"-collective_model": "packet"}), False)
    assert sim.run() == 0
    assert sim.collectives[0]["cycles"] == ev0[0]["cycles"]
    assert res[0][1]["insn"] == res[1][1]["insn"]


def _worker_params(rank, world, port, params, cases, q):
    import torch.distributed as dist
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ex = collectives.PacketExchange()
        out = [ex.run(params, kind, nbytes, 0, starts[rank])["finish_ps"] for kind, nbytes, starts in cases]
        q.put((rank, out, ex.stats))
    finally:
        dist.destroy_process_group()


def test_packet_exchange_four_ranks_overflow(native):
    """World size 4 with 2 KB slices: many packets per destination per epoch,
    so the fixed-slot exchange spills into its second all-to-all; results
    must still equal the single-process emulation exactly."""
    params = dict(PARAMS, slice_bytes=2048)
    cases = [("AllReduce", 1 << 20, [0, 0, 0, 0]), ("AllGather", 1 << 19, [0, 2_000_000, 0, 500_000]),
             ("ReduceScatter", 1 << 20, [0, 0, 0, 0]), ("AllToAll", 1 << 19, [0, 0, 7, 0]),
             ("Broadcast", 1 << 19, [0, 0, 0, 0])]
    res = _spawn(_worker_params, 4, params, cases)
    for i, (kind, nbytes, starts) in enumerate(cases):
        ref = collectives.emulate(params, kind, nbytes, starts)["finish_ps"]
        got = [res[r][1][i] for r in range(4)]
        assert got == ref, (kind, got, ref)
    st = res[0][2]
    # one fixed exchange per epoch, plus the spill exchanges
    assert st["exchanges"] > st["epochs"] > 0


def test_node_plan_places_apps_by_makespan(native, tmp_path, monkeypatch):
    """Whole-node mode: every application goes to the engine that minimises
    the step's makespan (GPU slots vs CPU cores, LPT inside each pool)."""
    from accel_sim_framework_distributed_amd.parallel.multi_gpu import DistributedSuite
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    apps = ["nn-rodinia-2.0-ft", "pathfinder-rodinia-2.0-ft", "backprop-rodinia-2.0-ft"]
    rodinia.generate_suite(str(tmp_path), apps)
    monkeypatch.setenv("ASIM_CPU_JOBS", "3")  # 1 GPU slot (no GPU here) + 2 CPU cores
    s = DistributedSuite(str(tmp_path), engine="node")
    t = {"nn-rodinia-2.0-ft": (0.1, 1.0), "pathfinder-rodinia-2.0-ft": (0.9, 0.5),
         "backprop-rodinia-2.0-ft": (0.2, 2.0)}  # (gpu, cpu) seconds
    for a, (g, c) in t.items():
        s.times[(a, "gpu")] = g
        s.times[(a, "cpu")] = c
    plan = s.plan()
    assert plan == {"nn-rodinia-2.0-ft": "gpu", "backprop-rodinia-2.0-ft": "gpu", "pathfinder-rodinia-2.0-ft": "cpu"}
    assert abs(s.predicted_span - 0.5) < 1e-9


def test_node_plan_prefers_gpu_among_equal_makespans(native, tmp_path, monkeypatch):
    """Plans with the shortest makespan (ASIM_NODE_GPU_TOLERANCE, default 0:
    exact ties): the one with the most applications on the GPU engine wins."""
    from accel_sim_framework_distributed_amd.parallel.multi_gpu import DistributedSuite
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    apps = ["nn-rodinia-2.0-ft", "pathfinder-rodinia-2.0-ft", "backprop-rodinia-2.0-ft"]
    rodinia.generate_suite(str(tmp_path), apps)
    monkeypatch.setenv("ASIM_CPU_JOBS", "9")
    s = DistributedSuite(str(tmp_path), engine="node")
    # backprop sets the span (1.0 s either way); nn and pathfinder are short
    # on both engines and fit on the GPU slot next to nothing else
    t = {"nn-rodinia-2.0-ft": (0.2, 0.1), "pathfinder-rodinia-2.0-ft": (0.3, 0.1), "backprop-rodinia-2.0-ft": (2.0, 1.0)}
    for a, (g, c) in t.items():
        s.times[(a, "gpu")] = g
        s.times[(a, "cpu")] = c
    plan = s.plan()
    assert abs(s.predicted_span - 1.0) < 1e-9
    assert plan == {"nn-rodinia-2.0-ft": "gpu", "pathfinder-rodinia-2.0-ft": "gpu", "backprop-rodinia-2.0-ft": "cpu"}


def test_node_widen_gives_threads_to_critical_cpu_app(native, tmp_path, monkeypatch):
    """Spare host cores go to the CPU-engine application on the critical path
    (-sim_cpu_threads), kept only while re-timing shows it scales; the plan
    list-schedules thread teams on the cores."""
    from accel_sim_framework_distributed_amd.parallel.multi_gpu import DistributedSuite
    from accel_sim_framework_distributed_amd.tracegen import rodinia
    apps = ["nn-rodinia-2.0-ft", "pathfinder-rodinia-2.0-ft", "backprop-rodinia-2.0-ft"]
    rodinia.generate_suite(str(tmp_path), apps)
    monkeypatch.setenv("ASIM_CPU_JOBS", "9")  # 1 GPU slot + 8 cores
    s = DistributedSuite(str(tmp_path), engine="node")
    base = {"nn-rodinia-2.0-ft": 0.1, "pathfinder-rodinia-2.0-ft": 0.3, "backprop-rodinia-2.0-ft": 1.0}
    scales = {"backprop-rodinia-2.0-ft": True, "pathfinder-rodinia-2.0-ft": False, "nn-rodinia-2.0-ft": False}
    for a, c in base.items():
        s.times[(a, "gpu")] = 5.0
        s.times[(a, "cpu")] = c

    def fake_run(app_kl, engine=None):
        a = app_kl[0]
        k = s.threads.get(a, 1)
        s.times[(a, engine)] = base[a] / (k ** 0.8 if scales[a] else 1.0)
        return a, 0, 0

    monkeypatch.setattr(s, "_run_app", fake_run)
    th = s.widen(max_threads=8)
    # backprop scales: 2 -> 4 -> 8 threads would need 8 + 2 cores; 4 fits
    # next to the two single-threaded apps... and 8 does not (8 + 1 + 1 > 8)
    assert th == {"backprop-rodinia-2.0-ft": 4}, th
    assert all(v == "cpu" for v in s.assignment.values())
    assert abs(s.predicted_span - 1.0 / 4 ** 0.8) < 1e-9
    # thread teams share the cores: two 4-thread jobs on 4 cores run back to back
    assert abs(DistributedSuite._cores_span([(1.0, 4), (1.0, 4)], 4) - 2.0) < 1e-12
    assert abs(DistributedSuite._cores_span([(1.0, 4), (1.0, 4)], 8) - 1.0) < 1e-12


# ---- data-parallel training step: collectives overlapping compute ----------
DP_KW = dict(layers=2, ctas=8, k_tiles=1, grad_mb=0.0625, straggle=0.6)
DP_EXTRA = {"-gpgpu_concurrent_kernel_sm": "1", "-collective_model": "packet", "-gpgpu_n_clusters": "16"}


def _dp_result(s):
    return (int(s.tot_cycle), [(k["uid"], k["start_cycle"], k["cycles"]) for k in s.kernels],
            [c["cycles"] for c in s.collectives])


def _dp_worker(rank, world, port, root, q):
    import torch.distributed as dist
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from accel_sim_framework_distributed_amd import _native
        from accel_sim_framework_distributed_amd.sim import build_args
        kl = os.path.join(root, f"rank{rank}", "kernelslist.g")
        import json
        extra = json.load(open(os.path.join(root, "extra.json")))
        s = _native.load().Simulator(build_args("QV100", kl, "cpu", extra), False)
        hook = collectives.PacketCollective()
        s.set_collective_hook(lambda d, now: hook(s, d, now))
        assert s.run() == 0
        q.put((rank, _dp_result(s), [e["mode"] for e in hook.events]))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("traffic", ["link_only", "mem_traffic"])
def test_dp_step_eight_ranks_match_in_process_emulation(native, tmp_path, traffic):
    """Eight gloo processes, one simulated GPU each, run unequal shards of a
    DDP step whose per-layer all-reduces (stream 2) overlap the backward pass
    (stream 1): every rank's kernel and collective timing equals the
    in-process emulation of all eight ranks (threads + linksim_run_local)
    exactly, and the collectives couple the ranks' clocks.  With
    -collective_mem_traffic the all-reduces' buffer traffic also runs through
    each rank's simulated memory system (RCCL copy kernels)."""
    import json
    import threading
    from accel_sim_framework_distributed_amd.sim import build_args
    from accel_sim_framework_distributed_amd.tracegen import training
    W = 8
    root = str(tmp_path / "dp")
    kls = training.write_dp_ranks(root, W, **DP_KW)
    extra = dict(DP_EXTRA, **({"-collective_mem_traffic": "1"} if traffic == "mem_traffic" else {}))
    with open(os.path.join(root, "extra.json"), "w") as f:
        json.dump(extra, f)
    res = _spawn(_dp_worker, W, root)
    assert all(m == ["rccl"] * DP_KW["layers"] for _, _, m in res)
    # oracle: all ranks in this process
    loc = collectives.LocalRanks(W)
    out = [None] * W

    def run(r):
        s = native.Simulator(build_args("QV100", kls[r], "cpu", extra), False)
        s.set_collective_hook(loc.hook(r, s))
        assert s.run() == 0
        out[r] = _dp_result(s)

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert [r[1] for r in res] == out
    # coupling: the fastest rank's first all-reduce waits for the slowest rank
    # (its collective lasts longer than the slowest rank's own)
    first = [r[1][2][0] for r in res]
    assert first[0] > first[-1]
    # overlap: backward kernels run back to back while the all-reduces proceed
    bwd = [k for k in res[0][1][1] if k[0] in (3, 4)]
    assert bwd[1][1] == bwd[0][1] + bwd[0][2]
    copies = [k for k in res[0][1][1] if k[0] >= 0x40000000]
    assert len(copies) == (DP_KW["layers"] if traffic == "mem_traffic" else 0)


@pytest.mark.slow
def test_bench_eight_gloo_ranks_dp_step_matches_local_ranks(native, tmp_path):
    """The driver's multi-GPU bench shape on the CPU tier: torchrun with 8
    ranks, ``bench.py --gpus 8 --engine cpu --dist-backend gloo`` (one
    simulated GV100 per rank, the DDP step's per-layer all-reduces exchanged
    as link packets every lookahead epoch, their buffer traffic through each
    rank's simulated L2/HBM).  Every rank's simulated DDP-step cycles equal
    the in-process emulation of all 8 ranks (threads + linksim_run_local)."""
    import json
    import subprocess
    import sys
    import threading
    from accel_sim_framework_distributed_amd.sim import build_args
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    W = 8
    tdir = tmp_path / "bench"
    env = dict(os.environ, OMP_NUM_THREADS="1", ASIM_CPU_JOBS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(W), "--engine", "cpu", "--dist-backend", "gloo", "--apps", "nn,dp-step",
           "--steps", "1", "--warmup", "0", "--trace-dir", str(tdir)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.split("\n") if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == W and out["metric"] == "sim KIPS (whole node)" and out["value"] > 0
    dp = out["dp_step"]
    assert dp["ranks"] == W and dp["collective_coupling"] == ["rccl"] and dp["collective_mem_traffic"]
    assert len(dp["simulated_cycles_per_rank"]) == W
    assert out["gpu_engine"]["apps_on_gpu"] == 0 and len(out["gpu_engine"]["kips_per_rank"]) == W
    # oracle: the same eight traces, all ranks in this process
    extra = {"-collective_model": "packet", "-gpgpu_concurrent_kernel_sm": "1", "-collective_mem_traffic": "1"}
    loc = collectives.LocalRanks(W)
    cyc = [None] * W
    kern = [None] * W

    def run(rk):
        s = native.Simulator(build_args("GV100", str(tdir / f"dp-step-{W}" / f"rank{rk}" / "kernelslist.g"), "cpu",
                                        extra), False)
        s.set_collective_hook(loc.hook(rk, s))
        assert s.run() == 0
        cyc[rk] = int(s.tot_cycle)
        kern[rk] = len(s.kernels)

    th = [threading.Thread(target=run, args=(rk,)) for rk in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert dp["simulated_cycles_per_rank"] == cyc
    assert dp["simulated_cycles_max_rank"] == max(cyc)
    # the collectives' copy kernels ran in every rank's simulated GPU
    assert dp["rank0_kernels"] == kern[0] > 9


def _loop_worker(rank, world, port, cases, q):
    import time
    import torch.distributed as dist
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = {}
        for mode in ("1", "0"):
            os.environ["ASIM_NATIVE_EXCHANGE"] = mode
            ex = collectives.PacketExchange()
            t = time.perf_counter()
            fin = [ex.run(PARAMS, kind, nbytes, 0, starts[rank])["finish_ps"] for kind, nbytes, starts in cases]
            out[mode] = (fin, dict(ex.stats), time.perf_counter() - t)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_native_exchange_loop_matches_python_loop_eight_ranks(native):
    """The C++ epoch loop (csrc/parallel/exchange.cc, over the c10d
    ProcessGroup) and the Python loop give identical finish times on 8 gloo
    ranks; the native loop ran (its stats say so) and is not slower."""
    from accel_sim_framework_distributed_amd import _native
    if _native.load_dist() is None:
        pytest.skip("_asim_dist not built")
    cases = [("AllReduce", 4 << 20, [0, 0, 0, 0, 0, 0, 0, 0]), ("AllGather", 2 << 20, [0, 900_000, 0, 0, 5, 0, 0, 0]),
             ("AllToAll", 1 << 20, [0] * 8)]
    res = _spawn(_loop_worker, 8, cases)
    for r, out in res:
        assert out["1"][0] == out["0"][0]
        assert out["1"][1].get("native") and out["1"][1]["epochs"] == out["0"][1]["epochs"] > 0
    ref = [collectives.emulate(PARAMS, k, b, s)["finish_ps"] for k, b, s in cases]
    for i in range(len(cases)):
        assert [res[r][1]["1"][0][i] for r in range(8)] == ref[i]


def test_cpu_share_is_one_gpus_share(monkeypatch):
    """A rank's host cores are one GPU's share of the node whether the node
    runs one rank or one per visible GPU (weak scaling keeps per-GPU
    resources fixed)."""
    from accel_sim_framework_distributed_amd.parallel import multi_gpu
    cls = next(v for v in vars(multi_gpu).values() if isinstance(v, type) and hasattr(v, "cpu_slots"))
    obj = cls.__new__(cls)
    monkeypatch.setenv("ASIM_CPU_JOBS", "0")
    monkeypatch.setattr(cls, "cgroup_cores", staticmethod(lambda: 64))
    monkeypatch.setattr(multi_gpu.os, "sched_getaffinity", lambda _: set(range(64)))
    for lws, gpus, want in (("1", 1, 64), ("1", 8, 8), ("8", 8, 8), ("4", 8, 8), ("2", 0, 32)):
        monkeypatch.setenv("LOCAL_WORLD_SIZE", lws)
        monkeypatch.setattr(cls, "visible_gpus", staticmethod(lambda g=gpus: g))
        assert obj.cpu_slots() == want, (lws, gpus)


def test_node_widen_offers_threads_to_the_gpu_critical_app(monkeypatch):
    """When the GPU side sets the node's span, its longest application is
    re-timed on a wider host thread team, and the plan moves it if that
    shortens the step (measured MI355X calibration times, round 4)."""
    from accel_sim_framework_distributed_amd.parallel import multi_gpu
    S = multi_gpu.DistributedSuite
    obj = S.__new__(S)
    cal = {"backprop": (0.0714, 0.1392), "bfs": (0.6649, 0.138), "heartwall": (0.2358, 0.1668),
           "hotspot": (0.164, 0.4031), "lud": (0.099, 0.0164), "nn": (0.0097, 0.0223), "nw": (0.207, 0.0294),
           "pathfinder": (0.037, 0.0093), "srad": (0.0355, 0.03), "streamcluster": (0.446, 0.0547),
           "dp-step": (0.1842, 0.1608)}
    dense = {"hotspot": 0.9, "dp-step": 0.85, "heartwall": 0.6, "backprop": 0.5}
    obj.apps = [(a, a) for a in cal]
    obj.times = {}
    for a, (g, c) in cal.items():
        obj.times[(a, "gpu")], obj.times[(a, "cpu")] = g, c
    obj.threads = {}
    obj._calibrating = False
    monkeypatch.setattr(S, "concurrency", lambda self: 2)
    monkeypatch.setattr(S, "cpu_slots", lambda self, reserve=0: 14)

    def run_app(self, app_kl, engine=None):  # thread-team scaling of the CPU engine
        a = app_kl[0]
        k = self.threads.get(a, 1)
        self.times[(a, engine)] = cal[a][1] / (k ** dense.get(a, 0.0))
    monkeypatch.setattr(S, "_run_app", run_app)
    obj.plan()
    before = obj.predicted_span
    assert obj.assignment["hotspot"] == "gpu"
    obj.widen()
    assert obj.predicted_span < 0.9 * before
    # the GPU keeps the applications it runs fastest
    assert sum(e == "gpu" for e in obj.assignment.values()) >= 3
    assert sum(obj.threads.get(a, 1) for a, e in obj.assignment.items() if e == "cpu") <= 14


@pytest.mark.slow
def test_bench_eight_gloo_ranks_node_mode_runs_rank0_plan(tmp_path):
    """``bench.py --engine node`` on 8 gloo ranks with the GPU engine mocked
    by the CPU engine (ASIM_MOCK_GPU=1): every rank calibrates under its own
    load, then all run rank 0's placement; the JSON carries every rank's
    plan, calibration and wall time (verdict r4 item 5)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    W = 8
    env = dict(os.environ, OMP_NUM_THREADS="1", ASIM_CPU_JOBS="2", ASIM_MOCK_GPU="1", ASIM_MOCK_GPU_SLOTS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(W), "--engine", "node", "--dist-backend", "gloo", "--apps", "nn,pathfinder",
           "--steps", "1", "--warmup", "0", "--trace-dir", str(tmp_path / "bench")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.split("\n") if ln.startswith("{")][-1])
    pr = out["per_rank"]
    assert [p["rank"] for p in pr] == list(range(W))
    assert out["plans_identical"] is True
    assert all(p["assignment"] == pr[0]["assignment"] and p["plan_source"] == "rank0" for p in pr)
    assert set(pr[0]["assignment"]) == {"nn-rodinia-2.0-ft", "pathfinder-rodinia-2.0-ft"}
    assert all(p["wall_s"] > 0 and p["insn"] > 0 and p["calibration_s"] for p in pr)
    assert out["wall_s_spread"]["max"] >= out["wall_s_spread"]["min"] > 0


def test_node_widen_tries_a_wider_team_when_doubling_does_not_pay(monkeypatch):
    """The dp step on an MI355X node's cores: 158 / 140 / 110 ms at 1 / 2 / 4
    threads (tools/dp_step_threads.py).  Two threads miss the 15 % bar, four
    clear it: widen() must keep four instead of giving up at two."""
    from accel_sim_framework_distributed_amd.parallel import multi_gpu
    S = multi_gpu.DistributedSuite
    obj = S.__new__(S)
    scale = {1: 0.158, 2: 0.140, 4: 0.110, 8: 0.105}
    cal = {"dp-step": (0.30, 0.158), "bfs": (0.50, 0.129), "hotspot": (0.16, 0.12)}
    obj.apps = [(a, a) for a in cal]
    obj.times = {}
    for a, (g, c) in cal.items():
        obj.times[(a, "gpu")], obj.times[(a, "cpu")] = g, c
    obj.threads = {}
    obj._calibrating = False
    monkeypatch.setattr(S, "concurrency", lambda self: 1)
    monkeypatch.setattr(S, "cpu_slots", lambda self, reserve=0: 14)

    def run_app(self, app_kl, engine=None):
        a = app_kl[0]
        k = self.threads.get(a, 1)
        self.times[(a, engine)] = scale[k] if a == "dp-step" else cal[a][1]
    monkeypatch.setattr(S, "_run_app", run_app)
    obj.plan()
    assert obj.assignment["dp-step"] == "cpu"
    obj.widen()
    assert obj.threads.get("dp-step") == 4
    assert obj.predicted_span < 0.135
