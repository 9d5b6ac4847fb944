"""L1 / L2 write policies and write-allocate modes (reference data_cache
wr_hit_* / wr_miss_*, gpu-cache.cc:1229-1599) on hand-built micro traces with
hand-computed hit/miss counts.  One warp writes one whole 128-byte line (four
fully written 32-byte sectors), then reads it back."""
import re

import numpy as np
import pytest

from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.tracegen import rodinia
from accel_sim_framework_distributed_amd.tracegen.builder import KernelBuilder

LINE = 0x7000_1000


def _kernel(kid, store=True, load=True):
    k = KernelBuilder(f"_Z2k{kid}Pi", (1, 1, 1), (32, 1, 1), nregs=16, kid=kid)
    base = np.full(k.g.nwarps, LINE, np.int64)
    if store:
        k.op("STG.E", [], [4, 5], base=base, stride=4)
    if load:
        k.op("LDG.E", [6], [4], base=base, stride=4)
        k.op("IADD3", [7], [6])
    k.op("EXIT")
    return k.build()


@pytest.fixture(scope="module")
def apps(tmp_path_factory):
    d = tmp_path_factory.mktemp("pol")
    return {"st_ld": rodinia.write_app(str(d / "st_ld"), [_kernel(1)], memcpy=False),
            "st_then_ld": rodinia.write_app(str(d / "two"), [_kernel(1, load=False), _kernel(2, store=False)],
                                            memcpy=False)}


def _run(native, kl, extra):
    s = native.Simulator(presets.args_for("QV100", extra) + ["-trace", kl, "-gpgpu_perf_sim_memcpy", "0"], False)
    assert s.run() == 0
    # a write-back L1 never drops a dirty victim: the LD/ST unit consumes a
    # fill reply only when the injection queue has room for its write-back
    assert "L1 write-backs lost" not in s.output
    return s.output


def _stat(out, key):
    m = re.findall(rf"{re.escape(key)} = ([0-9.]+)", out)
    return int(float(m[-1])) if m else 0


DL1 = "S:4:128:64,L:{wp}:m:{wa}:L,A:512:8,16:0,32"
DL2 = "S:32:128:24,L:B:m:{wa}:P,A:192:4,32:0,32"


def test_l1_lazy_write_allocate_makes_full_sectors_readable(native, apps):
    lazy = _run(native, apps["st_ld"], {"-gpgpu_cache:dl1": DL1.format(wp="T", wa="L")})
    noalloc = _run(native, apps["st_ld"], {"-gpgpu_cache:dl1": DL1.format(wp="T", wa="N")})
    # lazy fetch on read: the store allocates the line, the load hits it
    assert _stat(lazy, "Total_core_cache_stats_breakdown[GLOBAL_ACC_W][MISS]") == 1
    assert _stat(lazy, "Total_core_cache_stats_breakdown[GLOBAL_ACC_R][HIT]") == 1
    assert _stat(lazy, "Total_core_cache_stats_breakdown[GLOBAL_ACC_R][MISS]") == 0
    # no write-allocate: the load misses and fetches from the L2
    assert _stat(noalloc, "Total_core_cache_stats_breakdown[GLOBAL_ACC_R][MISS]") == 1
    assert _stat(noalloc, "Total_core_cache_stats_breakdown[GLOBAL_ACC_R][HIT]") == 0


def test_l1_write_back_absorbs_the_store(native, apps):
    wt = _run(native, apps["st_ld"], {"-gpgpu_cache:dl1": DL1.format(wp="T", wa="L")})
    wb = _run(native, apps["st_ld"], {"-gpgpu_cache:dl1": DL1.format(wp="B", wa="L")})
    # write-through sends the line's write to the L2, write-back keeps it dirty in L1
    assert _stat(wt, "L2_cache_stats_breakdown[GLOBAL_ACC_W][TOTAL_ACCESS]") == 1
    assert _stat(wb, "L2_cache_stats_breakdown[GLOBAL_ACC_W][TOTAL_ACCESS]") == 0
    assert _stat(wb, "Total_core_cache_stats_breakdown[GLOBAL_ACC_R][HIT]") == 1


def test_l1_fetch_on_write_of_partial_sectors_reads_the_line(native, tmp_path):
    # 2-byte stores cover half of each sector: fetch-on-write reads the line
    k = KernelBuilder("_Z2p1Pi", (1, 1, 1), (32, 1, 1), nregs=16)
    k.op("STG.E.U16", [], [4, 5], base=np.full(k.g.nwarps, LINE, np.int64), stride=4)
    k.op("EXIT")
    kl = rodinia.write_app(str(tmp_path / "p"), [k.build()], memcpy=False)
    f = _run(native, kl, {"-gpgpu_cache:dl1": DL1.format(wp="T", wa="F")})
    lz = _run(native, kl, {"-gpgpu_cache:dl1": DL1.format(wp="T", wa="L")})
    assert _stat(f, "L2_cache_stats_breakdown[GLOBAL_ACC_R][TOTAL_ACCESS]") >= 1
    assert _stat(lz, "L2_cache_stats_breakdown[GLOBAL_ACC_R][TOTAL_ACCESS]") == 0


def test_l2_no_write_allocate_sends_misses_to_dram(native, apps):
    # the first kernel's store reaches the L2 (L1 no-allocate), the second
    # kernel reads the line back: it hits in an allocating L2 only
    dl1 = DL1.format(wp="T", wa="N")
    lazy = _run(native, apps["st_then_ld"], {"-gpgpu_cache:dl1": dl1, "-gpgpu_cache:dl2": DL2.format(wa="L")})
    noal = _run(native, apps["st_then_ld"], {"-gpgpu_cache:dl1": dl1, "-gpgpu_cache:dl2": DL2.format(wa="N")})
    assert _stat(lazy, "L2_cache_stats_breakdown[GLOBAL_ACC_R][HIT]") == 1
    assert _stat(noal, "L2_cache_stats_breakdown[GLOBAL_ACC_R][HIT]") == 0
    assert _stat(noal, "L2_cache_stats_breakdown[GLOBAL_ACC_R][MISS]") == 1
