#!/usr/bin/env python3
"""One device-epoch-loop case at a time, with progress lines (locates a failing case)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ASIM_SEGV_TRACE", "1")
from accel_sim_framework_distributed_amd import _native  # noqa: E402
from accel_sim_framework_distributed_amd.parallel import collectives  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_device_exchange import CASES  # noqa: E402

ext = _native.load_dist()
for p, kind, nbytes, starts in CASES:
    print("case", kind, nbytes, len(starts), p["slice_bytes"], flush=True)
    ref = collectives.emulate(p, kind, nbytes, starts)["finish_ps"]
    r = ext.dev_run_local(p, kind, nbytes, 0, starts, 0)
    print("  ok" if list(r["finish_ps"]) == list(ref) else "  MISMATCH", r["epochs"], r["kernel_clocks_per_launch"], flush=True)
