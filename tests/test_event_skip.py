"""Event skipping is exact: quiet SM cycles inside an epoch, quiet memory-channel
ticks (requests riding the ROP / DRAM latency pipes) and whole quiet epochs
(epoch_decide's next-event fast-forward) are skipped with -sim_event_skip 1,
and every printed statistic must equal the cycle-by-cycle run (-sim_event_skip 0).
The reference simulates every cycle (gpgpu_sim::cycle, gpu-sim.cc:1871-2107);
this is the simulator-side analogue of its determinism requirement."""
import re

import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen import rodinia

WALL = re.compile(r"rate|slowdown|time|sec|skipped|epochs", re.I)


def _stats(out):
    """key = value lines without wall-clock / diagnostic ones."""
    kv = []
    for line in out.splitlines():
        m = re.match(r"^\s*([A-Za-z_][\w\[\]\.:\- ]*?)\s*=\s*(.+)$", line)
        if m and not WALL.search(m.group(1)):
            kv.append((m.group(1), m.group(2).strip()))
    return kv


def _run(native, kl, extra, config="QV100"):
    s = native.Simulator(presets.args_for(config, extra) + ["-trace", kl], False)
    assert s.run() == 0
    return s


APPS = {
    "streamcluster": lambda: rodinia.streamcluster(1024, 8, 3),
    "nw": lambda: rodinia.nw(48),
    "bfs": lambda: rodinia.bfs(1024, levels=3),
    "pathfinder": lambda: rodinia.pathfinder(500, 6, 5),
}


@pytest.mark.parametrize("app", sorted(APPS))
def test_event_skip_identical_stats(native, tmp_path, app):
    kl = rodinia.write_app(str(tmp_path / app), APPS[app]())
    on = _run(native, kl, {})
    off = _run(native, kl, {"-sim_event_skip": "0"})
    assert (on.tot_cycle, on.tot_insn) == (off.tot_cycle, off.tot_insn)
    a, b = _stats(on.output), _stats(off.output)
    assert len(a) > 50
    diff = [(x, y) for x, y in zip(a, b) if x != y]
    assert not diff and len(a) == len(b), diff[:5]
    # and skipping actually removed epochs
    assert sum(k["epochs"] for k in on.kernels) < sum(k["epochs"] for k in off.kernels)


def test_event_skip_identical_state(native, tmp_path):
    """Full architectural state after the run is byte-identical too."""
    kl = rodinia.write_app(str(tmp_path / "sc"), rodinia.streamcluster(1024, 8, 2))
    on = _run(native, kl, {"-gpgpu_perf_sim_memcpy": "0"})
    off = _run(native, kl, {"-gpgpu_perf_sim_memcpy": "0", "-sim_event_skip": "0"})
    a, b = bytearray(on.snapshot()), bytearray(off.snapshot())
    assert len(a) == len(b)
    # allowed to differ: the diagnostic count of skipped cycles, and what
    # depends on which epochs ran (gather scratch, mailbox-parity flags)
    n_sm, n_ch = 80, len(a) - 80 * native.sizeof_SMState
    n_ch //= native.sizeof_ChanState
    for base, size, fields in ((0, native.sizeof_SMState, native.epoch_dependent_SMState),
                               (n_sm * native.sizeof_SMState, native.sizeof_ChanState, native.epoch_dependent_ChanState)):
        for i in range(n_sm if base == 0 else n_ch):
            for off, n in fields:
                o = base + i * size + off
                a[o:o + n] = b[o:o + n] = bytes(n)
    assert a == b


def test_event_skip_intersim_topology(native, tmp_path):
    """-network_mode 1 topology (TITANX preset): per-pair interconnect latencies
    longer than the epoch, so packets stay in flight across several epochs."""
    kl = rodinia.write_app(str(tmp_path / "nw"), rodinia.nw(32))
    on = _run(native, kl, {}, "TITANX")
    off = _run(native, kl, {"-sim_event_skip": "0"}, "TITANX")
    assert (on.tot_cycle, on.tot_insn) == (off.tot_cycle, off.tot_insn)
    assert _stats(on.output) == _stats(off.output)
