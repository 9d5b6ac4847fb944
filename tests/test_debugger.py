"""Interactive timing debugger (reference gpgpu_debug, debug.cc:40-220;
g_single_step, gpu-sim.cc:1984-1990): single step, PC / cycle breakpoints,
memory-line watchpoints and pipeline dumps, driven by a command script."""
import os
import re

import pytest

from accel_sim_framework_distributed_amd.sim import build_args
from accel_sim_framework_distributed_amd.tracegen import rodinia


def _trace(tmp_path):
    kl = rodinia.write_app(str(tmp_path / "va"), [rodinia.vectoradd(4096)], text=True)
    txt = open(os.path.join(os.path.dirname(kl), "kernel-1.traceg")).read()
    pc = next(ln.split()[0] for ln in txt.split("\n") if " DADD " in ln)
    return kl, int(pc, 16)


def _run(native, kl, script, extra=None):
    args = build_args("QV100", kl, "cpu", dict({"-sim_debug": "1", "-sim_debug_script": str(script)}, **(extra or {})))
    s = native.Simulator(args, False)
    rc = s.run()
    return rc, s


def test_breakpoint_watchpoint_step_and_dump(native, tmp_path):
    kl, pc = _trace(tmp_path)
    store_line = rodinia.buf(2)  # c[] of vectoradd: the STG target
    script = tmp_path / "dbg.txt"
    script.write_text("\n".join([
        "h",
        f"b {pc:x}",            # DADD issued (any SM)
        "c",
        "dp",                   # pipelines of the busy SMs at the breakpoint
        "i",
        "d 1",
        f"w {store_line + 8:x}",  # the first line of c[]
        "c",
        "l",
        "s 3",
        "q",
    ]) + "\n")
    rc, s = _run(native, kl, script)
    out = s.output
    m = re.search(r"breakpoint 1 hit: core (\d+) warp (\d+) issued pc 0x([0-9a-f]+) at cycle (\d+)", out)
    assert m and int(m.group(3), 16) == pc, out[-3000:]
    dump = out.split("(asim debugger) dp", 1)[1][:2000]
    assert f"SM {m.group(1)}" in dump, dump
    m2 = re.search(r"watchpoint 2 hit: core \d+ sends a request for line 0x([0-9a-f]+)", out)
    assert m2 and int(m2.group(1), 16) == store_line & ~127, out[-3000:]
    # the watchpoint fired after the breakpoint, and 3 steps later the user stopped
    assert int(re.search(r"watchpoint 2 hit: .* at cycle (\d+)", out).group(1)) >= int(m.group(4))
    assert "simulation stopped by the user" in out and "exit detected" in out
    # stopping early: the kernel ended with the stop (like -gpgpu_max_cycle)
    assert s.tot_cycle < _full_cycles(native, kl)


def _full_cycles(native, kl):
    s = native.Simulator(build_args("QV100", kl, "cpu"), False)
    assert s.run() == 0
    return s.tot_cycle


def test_break_cycle_then_script_end_runs_to_completion(native, tmp_path):
    """-sim_break_cycle stops once at a cycle (reference g_single_step); when
    the script ends the run continues, and the results equal an undebugged run."""
    kl, _ = _trace(tmp_path)
    script = tmp_path / "s.txt"
    script.write_text("i\ns 2\ni\n")
    rc, s = _run(native, kl, script, {"-sim_break_cycle": "2000"})
    assert rc == 0
    stops = [int(x) for x in re.findall(r"stopped at cycle (\d+)", s.output)]
    assert len(stops) == 2 and 2000 <= stops[0] < stops[1]
    assert s.tot_cycle == _full_cycles(native, kl)
    # a cycle breakpoint set from the script fires once
    script.write_text("bc 3000\nc\nl\n")
    rc, s = _run(native, kl, script)
    assert re.search(r"breakpoint 1 hit: cycle 3000 reached \(now (\d+)\)", s.output)
    assert "(hits 1)" in s.output
