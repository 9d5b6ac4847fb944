"""Device-resident epoch loop of the packet collective (csrc/parallel/
linksim_dev.hip, exchange.cc exchange_run_device / dev_run_local).

The ranks' LinkSim states live in HBM and one epoch kernel per epoch delivers
the last all-to-all's slots and packs the next epoch's packets; the results
must equal the host model's in-process emulation (linksim_run_local) bit for
bit, including epochs where a rank sends more than the fixed slot holds (the
overflow exchange).  RCCL refuses two ranks on one GPU, so the multi-rank
cases run every rank in one process: with the transposition kernel as the
all-to-all, and with a 1-rank RCCL group's all-to-all of all ranks' buffers
(loopback: the per-epoch work of an 8-GPU run on one MI355X).
"""
import os
import socket

import pytest

from accel_sim_framework_distributed_amd.parallel import collectives

PARAMS = dict(link_gbps=153.0, latency_ns=1000.0, links=7, slice_bytes=65536, max_channels=16, reduce_gbps=900.0)
# 64-byte slices: hundreds of packets per destination in one epoch -> overflow exchanges
SMALL = dict(PARAMS, slice_bytes=64)

CASES = [
    (PARAMS, "AllReduce", 8 << 20, [0] * 8),
    (PARAMS, "AllReduce", 4 << 20, [0, 3_000_000, 0, 0, 17, 0, 900_000, 0]),
    (PARAMS, "AllGather", 2 << 20, [0, 900_000, 0, 0, 5, 0, 0, 0]),
    (PARAMS, "ReduceScatter", 4 << 20, [0] * 4),
    (PARAMS, "Broadcast", 4 << 20, [0, 0, 0, 0, 0]),
    (PARAMS, "Reduce", 2 << 20, [0, 0, 1_000_000]),
    (PARAMS, "AllToAll", 1 << 20, [0] * 8),
    (PARAMS, "SendRecv", 1 << 20, [0, 2_000_000]),
    (SMALL, "AllReduce", 1 << 20, [0] * 8),
    (SMALL, "AllToAll", 256 << 10, [0, 0, 4_000_000, 0]),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ext():
    from accel_sim_framework_distributed_amd import _native
    ext = _native.load_dist()
    if ext is None:
        raise RuntimeError("_asim_dist (device epoch loop) is not built: run build_native.py")
    return ext


@pytest.mark.gpu
def test_device_loop_matches_host_emulation():
    ext = _ext()
    for p, kind, nbytes, starts in CASES:
        ref = collectives.emulate(p, kind, nbytes, starts)["finish_ps"]
        r = ext.dev_run_local(p, kind, nbytes, 0, starts, 0)
        assert list(r["finish_ps"]) == list(ref), (kind, nbytes, starts)
        assert r["epochs"] > 0


@pytest.mark.gpu
def test_device_loop_over_rccl_loopback_and_one_rank_exchange():
    """The same cases with a 1-rank RCCL group carrying all ranks' buffers,
    and PacketExchange on that group taking the device-resident path."""
    import torch
    import torch.distributed as dist
    ext = _ext()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        pg = dist.distributed_c10d._get_default_group()
        for p, kind, nbytes, starts in CASES:
            ref = collectives.emulate(p, kind, nbytes, starts)["finish_ps"]
            r = ext.dev_run_local(p, kind, nbytes, 0, starts, 0, pg)
            assert list(r["finish_ps"]) == list(ref), (kind, nbytes, starts)
        # the exchange driver itself on the 1-rank group: one epoch, device loop
        ex = collectives.PacketExchange()
        out = ex.run(PARAMS, "AllReduce", 8 << 20, 0, 1234)
        assert out["finish_ps"] == 1234 and ex.stats.get("device_loop") and ex.stats["epochs"] == 1
    finally:
        dist.destroy_process_group()


def _gloo_dev_worker(rank, world, port, cases, q):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    torch.cuda.set_device(0)
    import datetime
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120))
    try:
        ex = collectives.PacketExchange(device=torch.device("cuda", 0))
        out = [ex.run(p, kind, nbytes, 0, starts[rank])["finish_ps"] for p, kind, nbytes, starts in cases]
        q.put((rank, out, dict(ex.stats)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_device_loop_multi_rank_over_gloo_device_tensors():
    """The multi-rank driver of the device loop (exchange_run_device: batched
    epochs, the global stop, the overflow all-to-all from the device buffer)
    with 4 real ranks on one MI355X.  RCCL refuses two ranks on one GPU, so the
    all-to-alls of the device buffers go over gloo here; the 8-GPU node runs
    the same driver over RCCL."""
    import torch.multiprocessing as mp
    _ext()
    cases = [c for c in CASES if len(c[3]) == 4] + [(PARAMS, "AllReduce", 4 << 20, [0, 700_000, 0, 13]),
                                                     (SMALL, "AllGather", 128 << 10, [0, 0, 0, 2_000_000])]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_dev_worker, args=(r, 4, port, cases, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, (p, kind, nbytes, starts) in enumerate(cases):
        ref = collectives.emulate(p, kind, nbytes, starts)["finish_ps"]
        assert [res[r][1][i] for r in range(4)] == list(ref), (kind, nbytes, starts)
    for r in range(4):
        assert res[r][2].get("device_loop") and res[r][2]["exchanges"] >= res[r][2]["epochs"] > 0
