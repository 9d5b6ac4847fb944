#!/usr/bin/env python3
"""Entry point at the reference's path (util/plotting/merge-stats.py); implementation in
accel_sim_framework_distributed_amd.plotting.merge_stats."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from accel_sim_framework_distributed_amd.plotting.merge_stats import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
