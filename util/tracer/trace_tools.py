#!/usr/bin/env python3
"""Entry point (util/tracer/trace_tools.py): generate | convert | info |
occupancy | bbv -- implementation in accel_sim_framework_distributed_amd.tracegen.cli."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from accel_sim_framework_distributed_amd.tracegen.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
