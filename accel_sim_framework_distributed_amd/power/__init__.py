"""AccelWattch-compatible power modelling utilities.

* ``xmlcfg``    -- read / write AccelWattch XML (``<param name= value=/>``)
  files, default XMLs for this framework's presets;
* ``report``    -- parse ``accelwattch_power_report.log`` written by the
  simulator (reference print_power_kernel_stats,
  accelwattch/gpgpu_sim_wrapper.cc:974-1041);
* ``calibrate`` -- bounded, constrained least squares (the QP of the
  reference's util/accelwattch/quadprog_solver.m) fitting per-component
  scaling factors to measured hardware power, MAPE / error metrics, and
  re-scaling an XML with the fitted factors;
* ``hwpower``   -- hardware power capture on MI355X via amd-smi / rocm-smi
  (the reference's NVML measureGpuPower.cpp).
"""
from .xmlcfg import read_xml, write_xml, default_params  # noqa: F401
from .report import parse_power_report  # noqa: F401
from .calibrate import fit_scaling, mape, apply_factors  # noqa: F401
