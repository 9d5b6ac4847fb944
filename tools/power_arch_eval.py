#!/usr/bin/env python3
"""What-if: the power suite's held-out fit with the architectural energy model
(csrc/power/arch_energy.cc) in place of the fixed per-access table.  The
saved validation record holds per-component powers; components fed by one
activity are rescaled exactly, multi-activity ones (DCP, ICP, CCP, RFP, L2CP,
DRAMP) by the mean energy ratio of their activities (an approximation)."""
import json, sys, numpy as np
sys.path.insert(0,'/root/repo')
from accel_sim_framework_distributed_amd import _native
from accel_sim_framework_distributed_amd.models import presets
from accel_sim_framework_distributed_amd.power import calibrate, mi355x_validation as mv
m=_native.load()
d=json.load(open('/root/repo/profiles/power_mi355x_validation_r4.json'))
A=np.asarray(d['components_w']); b=np.asarray(d['measured_w'])
names=m.PowerModel.activity_names()
tab={n:m.PowerModel.base_nj(i) for i,n in enumerate(names)}
cmp_of={'TOT_INST':'IBP','FP_INT':'SCHEDP','IC_H':'ICP','IC_M':'ICP','DC_RH':'DCP','DC_RM':'DCP','DC_WH':'DCP','DC_WM':'DCP','CC_H':'CCP','CC_M':'CCP','SHRD_ACC':'SHRDP','REG_RD':'RFP','REG_WR':'RFP','INT_ACC':'INTP','FP_ACC':'FPUP','DP_ACC':'DPUP','INT_MUL_ACC':'INT_MULP','FP_MUL_ACC':'FP_MULP','FP_SQRT_ACC':'FP_SQRTP','FP_LG_ACC':'FP_LGP','FP_SIN_ACC':'FP_SINP','FP_EXP_ACC':'FP_EXP','DP_MUL_ACC':'DP_MULP','TENSOR_ACC':'TENSORP','TEX_ACC':'TEXP','MEM_RD':'DRAMP','MEM_WR':'DRAMP','MEM_PRE':'MCP','L2_RH':'L2CP','L2_RM':'L2CP','L2_WH':'L2CP','L2_WM':'L2CP','NOC_A':'NOCP','PIPE_A':'PIPEP'}
args=presets.args_for("MI355X",{})
for node,dram in ((3.0,2.5),(5.0,2.5),(7.0,3.9)):
  arch=m.arch_energy(args,node_nm=node,dram_pj_per_bit=dram,tensor_macs_per_lane=128.0)['base_nj']
  ratio={}
  for a,c in cmp_of.items():
    ratio.setdefault(c,[]).append(arch[a]/tab[a])
  comps=d['components']
  A2=A.copy()
  for j,c in enumerate(comps):
    if c in ratio: A2[:,j]*=np.mean(ratio[c])
  for label,AA in (("table",A),(f"arch {node}nm",A2)):
    s=mv.fit_heldout(AA,b,d['kernels'],d['measured_sclk_mhz'],d['measured_vddgfx_mv'],d['power_cap_w'],d['max_sclk_mhz'])
    print(f"{label:12s} uncal(all) {calibrate.mape(AA.sum(1),b)[0]:6.2f} heldout {s['mape_heldout']:6.2f} uncal_heldout {s['mape_heldout_uncalibrated']:6.2f} insample {s['mape_calibration_in_sample']:6.2f} bound {s['factors_at_bound']}", {k:round(v,2) for k,v in s['group_factors'].items()})
