// AccelWattch-compatible power model.
//
// Reads the same XML schema as the reference (<param name=... value=.../>:
// per-activity dynamic scaling factors, constant / idle-SM power and the
// categorical first-lane / additional-lane static powers; reference
// gpgpu_sim_wrapper.cc:534-971, configs/tested-cfgs/*/accelwattch_*.xml).
// McPAT/CACTI (~49 kLoC in the reference) only supplies per-access base
// energies at init time; here those are a fixed per-activity energy table
// (csrc/power/power.cc), so a power sample is a small linear model:
//   P = constant + idle_sm * n_idle + static(category, lanes)
//       + sum_i  base_nJ[i] * scale[i] * accesses[i] / t
// which the GPU engine evaluates for all SMs x samples as one matrix
// product (counters x coefficients) and the host evaluates per kernel.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../model/mem.h"

namespace asim {

enum PwrAct : int {
  PA_TOT_INST = 0, PA_FP_INT, PA_IC_H, PA_IC_M, PA_DC_RH, PA_DC_RM, PA_DC_WH, PA_DC_WM, PA_CC_H, PA_CC_M,
  PA_SHRD_ACC, PA_REG_RD, PA_REG_WR, PA_INT_ACC, PA_FP_ACC, PA_DP_ACC, PA_INT_MUL_ACC, PA_FP_MUL_ACC,
  PA_FP_SQRT_ACC, PA_FP_LG_ACC, PA_FP_SIN_ACC, PA_FP_EXP_ACC, PA_DP_MUL_ACC, PA_TENSOR_ACC, PA_TEX_ACC,
  PA_MEM_RD, PA_MEM_WR, PA_MEM_PRE, PA_L2_RH, PA_L2_RM, PA_L2_WH, PA_L2_WM, PA_NOC_A, PA_PIPE_A, PA_COUNT
};
extern const char* const kPwrActName[PA_COUNT];

struct Activity {
  double a[PA_COUNT] = {};
  double cycles = 0;        // core cycles of the sample
  double idle_sms = 0;      // average idle SMs
  double avg_lanes = 0;     // average active threads per warp instruction
  double voltage = 1.0;
  // unit mix flags for the static category
  bool int_used = false, fp_used = false, dp_used = false, sfu_used = false, tex_used = false, tensor_used = false;
};

struct PowerReport {
  double dynamic_w[PA_COUNT] = {};
  double dynamic = 0;
  double static_w = 0;
  double constant = 0;
  double idle = 0;
  double total = 0;
  std::string static_category;
};

class PowerModel {
 public:
  // mode: 0 SIM (simulated activity), 1 HW (activity from hw_perf.csv),
  // 2 HYBRID (hw for selected counters)
  bool load_xml(const std::string& path, std::string* err = nullptr);
  void set_param(const std::string& k, double v) { p_[k] = v; }
  double param(const std::string& k, double dflt = 0) const;
  PowerReport compute(const Activity& act, double core_mhz, uint32_t n_sm) const;
  // activity of one kernel from stat deltas
  static Activity activity_from_stats(const std::vector<SMStats>& dsm, const std::vector<MemStats>& dmem,
                                      uint64_t cycles);
  // hw_perf.csv row -> activity (HW mode); returns false if not found
  static bool activity_from_hw_csv(const std::string& csv, const std::string& bench, const std::string& kernel,
                                   Activity& out, uint32_t n_sm);
  static double base_nj(int act);
  // coefficient vector (W per access-per-cycle at 1 MHz) for matrix evaluation
  std::vector<double> coefficients(double core_mhz) const;

 private:
  std::map<std::string, double> p_;
};

}  // namespace asim
