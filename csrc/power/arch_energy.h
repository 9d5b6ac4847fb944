// Architectural energy model: the per-access base energies of the power
// model derived from the simulated machine's geometry and a technology node,
// the role McPAT (component tree) and CACTI (array models) play at init time
// in the reference (gpgpu-sim/src/accelwattch: Processor::compute
// processor.cc:482, Core core.h:77-260, cacti Ucache.cc:731 design-space
// search; SURVEY §2.6 "McPAT core" / "CACTI": CPU init-time constants).
//
// Arrays (caches, shared memory, register file, instruction buffer) go
// through a first-order SRAM model: the data and tag arrays are split into
// subarrays by an exhaustive search over wordline / bitline divisions and sets
// per wordline, minimising energy x delay (CACTI's search), and a read or a
// write is priced as wordline + bitline swing + sense amplifiers + decoder +
// H-tree wires.  Logic (ALUs, scheduler, pipeline registers) is priced per
// operation from 45 nm reference energies scaled by feature size and Vdd^2;
// the interconnect per flit from the wire length across the estimated die;
// DRAM per bit.  The result replaces power.cc's fixed energy table when the
// XML sets <param name="energy_model" value="1"/>; the XML scaling factors
// (calibration) then apply on top, as in AccelWattch.
#pragma once
#include <string>
#include <vector>

#include "../model/config.h"
#include "power_eval.h"

namespace asim {

// device parameters of one technology node (high-performance logic,
// interpolated in log(feature size) between tabulated nodes)
struct TechParams {
  double node_nm = 12;
  double vdd = 0.8;          // nominal supply (V)
  double c_gate = 0.85;      // gate capacitance per um of width (fF/um)
  double c_wire = 0.18;      // intermediate-layer wire capacitance (fF/um)
  double i_leak = 60;        // subthreshold leakage per um of width (nA/um)
  double sram_cell_um2 = 0.06;
  static TechParams for_node(double node_nm, double vdd_override = 0.0);
};

struct ArrayGeom {
  const char* name = "";
  double bytes = 0;        // data capacity
  uint32_t line_bytes = 0; // bytes per line (one row of the logical array per way)
  uint32_t assoc = 1;      // ways (1: a plain RAM)
  uint32_t out_bits = 0;   // bits delivered per read (and written per write)
  uint32_t tag_bits = 0;   // 0: no tag array (RAM)
  uint32_t banks = 1;      // independent banks (one is accessed per access)
  bool sequential = true;  // tag first, then only the hit way's data (else all ways read)
};

struct ArrayResult {
  std::string name;
  double e_read_nj = 0, e_write_nj = 0, e_tag_nj = 0;
  double leak_w = 0, area_mm2 = 0, t_access_ns = 0;
  uint32_t ndwl = 0, ndbl = 0, nspd = 0, sub_rows = 0, sub_cols = 0;
};

ArrayResult model_array(const ArrayGeom& g, const TechParams& t);

struct ArchEnergyParams {
  double node_nm = 12;
  double vdd = 0;                // 0: the node's nominal
  double dram_pj_per_bit = 3.9;  // HBM2 class; HBM3E ~2.5
  double dram_act_nj = 0.9;      // row activate + precharge
  double tensor_macs_per_lane = 0;  // 0: 32 for 32-wide warps, 128 for 64-wide waves
};

struct ArchEnergy {
  double base_nj[PA_COUNT] = {};
  std::vector<ArrayResult> arrays;
  double sm_area_mm2 = 0, l2_area_mm2 = 0, die_mm2 = 0;
  double leak_sm_w = 0, leak_l2_w = 0;  // array leakage (informational; static power stays in the XML)
  TechParams tech;
};

ArchEnergy arch_energy(const SimCfg& c, const ArchEnergyParams& p);
std::string arch_energy_report(const ArchEnergy& e);

}  // namespace asim
