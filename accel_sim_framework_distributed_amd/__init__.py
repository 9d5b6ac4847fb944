"""accel-sim-framework-distributed, rebuilt MI355X-native.

A trace-driven cycle-level GPU performance + power simulator (the capabilities
of Accel-Sim / GPGPU-Sim / AccelWattch and the "distributed" NCCL fork) whose
cycle engine runs ON an MI355X: one CDNA4 wavefront simulates one SM or one
memory channel, state resident in LDS, one grid barrier per PDES epoch; a
bit-identical CPU reference engine runs the same single-source model.

Subpackages
  models/        simulated-GPU presets (gpgpusim.config/trace.config writers)
  ops/           the HIP engine front-end and device micro-benchmarks
  parallel/      multi-GPU simulation over RCCL, job-level parallel runners
  tracegen/      synthetic traces (Rodinia-2.0-ft shaped), trace formats
  job_launching/ run_simulations / job_status / monitor / get_stats / procman
  plotting/      correlator (sim vs HW), stat plots
  tuner/         microbenchmark-driven config tuner
  power/         AccelWattch calibration (quadratic programming)
  utils/         stats parsing, helpers
"""
__version__ = "0.1.0"

import os as _os

# The GPU engine runs one kernel per in-flight simulation, each on its own
# stream.  HIP gives a process 4 hardware queues by default, and kernels of
# streams that share a queue run one after another: a GV100 plan keeps 6
# simulations in flight (profiles/r6/README.md, "Hardware queues": GPU-engine
# suite +30 %, sweep +55 % at 8 queues).  ASIM_GPU_HW_QUEUES (default 8, 0:
# leave the variable alone) raises GPU_MAX_HW_QUEUES to at least that many;
# takes effect when the package is imported before the process's first HIP
# call.


def _raise_hw_queues() -> None:
    try:
        want = int(_os.environ.get("ASIM_GPU_HW_QUEUES", "8") or 0)
        have = int(_os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)
    except ValueError:
        return
    if want > 0 and have < want:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(min(want, 32))


_raise_hw_queues()

from .sim import SimResult, Simulator, simulate  # noqa: F401,E402
