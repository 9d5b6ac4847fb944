#!/usr/bin/env python3
"""Validate the simulator's stand-in for RCCL's library kernels against the
hardware counters of the real ones (verdict r3 item 6; reference: NVBit traces
NCCL's own kernels, util/tracer_nvbit/tracer_tool/tracer_tool.cu:380-506).

On a 1-rank communicator (the only one a one-GPU box allows: RCCL refuses two
ranks on one device) ncclAllReduce of the example's 32 Mi floats runs as the
HIP runtime's blit kernel ``__amd_rocclr_copyBuffer`` (the library kernel that
moves the payload; profiles/rccl_trace/dispatches.csv).  With
``-collective_mem_traffic`` the simulator runs the same payload movement as
``make_copy_kernel`` (csrc/trace/trace.cc): 16 B-per-lane loads and stores
over ``-collective_max_channels`` workgroups.  This script

1. reads the rocprofv3 counters of every ``copyBuffer`` dispatch of the
   example (tools/archive/gpu_r4_rccl.sh: SQ_INSTS_*, SQ_WAVES, TCC_REQ / TCC_HIT /
   TCC_EA0_RDREQ / TCC_EA0_WRREQ);
2. simulates the stand-in for the same bytes with the tuned MI355X config
   (a 2-rank all-reduce command moves 2(n-1)/n x S = S bytes each way, the
   1-rank copy's volume) and reads its statistics;
3. compares the vector-memory instruction counts and the L2 request / fabric
   traffic, and writes profiles/r4/rccl_copy_validation.json.

    python tools/rccl_validate.py [gpurun_out/r4rccl]
"""
from __future__ import annotations

import json
import os
import re
import sqlite3
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COUNT = 32 * 1024 * 1024  # floats per rank (examples/all-reduce/main.hip)


def hw_counters(d: str):
    """copyBuffer dispatches of the example: counters summed over them, and
    the per-dispatch grid/workgroup shapes."""
    tot, shapes, disp = {}, set(), set()
    for p in ("p1", "p2", "p3"):
        dbs = [os.path.join(r, f) for r, _, fs in os.walk(os.path.join(d, p)) for f in fs if f.endswith(".db")]
        for db in dbs:
            c = sqlite3.connect(db)
            for name, cnt, val, did, gx, wx in c.execute(
                    "select kernel_name, counter_name, value, dispatch_id, grid_size, workgroup_size "
                    "from counters_collection"):
                if "copyBuffer" not in name:
                    continue
                tot[cnt] = tot.get(cnt, 0.0) + float(val)
                shapes.add((int(gx), int(wx)))
                disp.add((p, did))
    return tot, sorted(shapes), len(disp)


def hw_durations(d: str):
    """copyBuffer dispatches per counter pass: count, shapes, summed duration"""
    out = {}
    for p in ("p1", "p2", "p3"):
        dbs = [os.path.join(r, f) for r, _, fs in os.walk(os.path.join(d, p)) for f in fs if f.endswith(".db")]
        for db in dbs:
            c = sqlite3.connect(db)
            rows = list(c.execute("select duration, grid_x, workgroup_x from kernels where name like '%copyBuffer%'"))
            out[p] = dict(dispatches=len(rows), busy_us=round(sum(r[0] for r in rows) / 1e3, 1),
                          shapes=sorted({(int(r[1]), int(r[2])) for r in rows}))
    return out


def simulate_standin():
    from accel_sim_framework_distributed_amd import _native
    from accel_sim_framework_distributed_amd.sim import build_args
    d = tempfile.mkdtemp(prefix="asim_rccl_")
    kl = os.path.join(d, "kernelslist.g")
    with open(kl, "w") as f:
        f.write(f"ncclAllReduce,count={COUNT},datatype=float,op=sum,nranks=2\n")
    s = _native.load().Simulator(build_args("MI355X", kl, "cpu", {"-collective_mem_traffic": "1",
                                                                 "-collective_model": "ring"}), False)
    assert s.run() == 0, s.output[-2000:]
    out = s.output
    def last(key):
        m = re.findall(rf"^\s*{re.escape(key)}\s*=\s*([0-9.]+)", out, re.M)
        return float(m[-1]) if m else None
    def l2(kind, outcome):
        m = re.findall(rf"L2_cache_stats_breakdown\[{kind}\]\[{outcome}\] = (\d+)", out)
        return float(m[-1]) if m else 0.0
    # the simulator prints the SQ counter classes as gpgpu_n_<class>_insn
    st = {f"SQ_INSTS_{k.upper()}": last(f"gpgpu_n_{k}_insn") for k in ("valu", "salu", "smem", "vmem_rd", "vmem_wr",
                                                                        "lds")}
    st["SQ_INSTS_BRANCH"] = last("gpgpu_n_sq_branch_insn")
    st["gpgpu_n_tot_w_icount"] = last("gpgpu_n_tot_w_icount")
    st["L2_read_accesses"] = l2("GLOBAL_ACC_R", "TOTAL_ACCESS")
    st["L2_write_accesses"] = l2("GLOBAL_ACC_W", "TOTAL_ACCESS")
    st["L2_read_hits"] = l2("GLOBAL_ACC_R", "HIT")
    st["kernels"] = [dict(name=k["name"], cycles=k["cycles"]) for k in s.kernels]
    return st, out


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "r4rccl")
    hw, shapes, ndisp = hw_counters(d)
    sim, out = simulate_standin()
    res = dict(hardware=dict(kernel="__amd_rocclr_copyBuffer (RCCL 1-rank all-reduce payload copy)",
                             dispatches_over_passes=ndisp, grid_and_workgroup=shapes, counters=hw,
                             dispatch_time_per_pass=hw_durations(d)),
               standin=dict(kernel="make_copy_kernel (-collective_mem_traffic)", stats=sim))
    cmp = {}
    def ratio(a, b):
        return None if not a or b is None else round(b / a, 4)
    # vector-memory instructions: exact volumes of the copy
    cmp["VMEM_RD"] = ratio(hw.get("SQ_INSTS_VMEM_RD"), sim.get("SQ_INSTS_VMEM_RD"))
    cmp["VMEM_WR"] = ratio(hw.get("SQ_INSTS_VMEM_WR"), sim.get("SQ_INSTS_VMEM_WR"))
    # L2 traffic: requests in, fabric reads / writes out (64 B TCC requests)
    if hw.get("TCC_REQ_sum"):
        cmp["L2_requests"] = ratio(hw["TCC_REQ_sum"], (sim["L2_read_accesses"] or 0) + (sim["L2_write_accesses"] or 0))
    res["sim_over_hw"] = cmp
    res["note"] = ("Ratios sim/hw; within 0.9-1.1 counts as matching.  ALU counts are not compared: the stand-in "
                   "moves bytes only, the blit kernel also computes addresses (its VALU/SALU are listed).  Time is "
                   "not compared: on one rank RCCL moves the payload as ~256 small blit dispatches (~3 us each, "
                   "launch-bound, dispatch_time_per_pass), while the stand-in models the multi-rank collective "
                   "kernel's single persistent launch over -collective_max_channels workgroups; the 1-rank "
                   "communicator is the only one a one-GPU box can run.")
    os.makedirs(os.path.join(ROOT, "profiles", "r4"), exist_ok=True)
    p = os.path.join(ROOT, "profiles", "r4", "rccl_copy_validation.json")
    json.dump(res, open(p, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
