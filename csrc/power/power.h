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
// evaluated on the host per sample from the engines' activity counters.
// DVFS (reference gpgpu_sim_wrapper.cc:948-958 scales static power by the
// voltage ratio and dynamic power by its square; -dvfs_enabled): with a
// `power_cap` parameter -- the package power limit MEASURED by amd-smi
// (power_suite measure), not fitted -- the simulator's governor picks for the
// next sample the highest core clock ratio s in [dvfs_min_clock_ratio, 1]
// whose power fits under the cap, with the rail voltage on the line
//   V(s) / V(1) = dvfs_v_floor + (1 - dvfs_v_floor) * s
// (dvfs_v_floor from the measured clock / voltage pairs).  At ratio s the
// core-domain dynamic power is  base * accesses-per-cycle * f(s) * V(s)^2,
// static and idle-core power scale with V(s), DRAM power keeps the HBM rail's
// voltage, and the slower clock makes the sample's cycles longer in simulated
// time (Engine::set_core_clock).  A sample above the cap is reported as it is.
#pragma once
#include <map>
#include <ostream>
#include <string>
#include <vector>

#include "../model/mem.h"
#include "power_eval.h"

namespace asim {

extern const char* const kPwrActName[PA_COUNT];

struct Activity {
  double a[PA_COUNT] = {};
  double cycles = 0;        // core cycles of the sample
  double idle_sms = 0;      // average idle SMs
  double avg_lanes = 0;     // average active threads per warp instruction
  double issue_frac = -1;   // SM-cycles with an issue / (SMs x cycles); < 0: unknown (the residency fraction)
  double voltage = 1.0;
  // unit mix flags for the static category
  bool int_used = false, fp_used = false, dp_used = false, sfu_used = false, tex_used = false, tensor_used = false;
};

extern const char* const kPwrCmpName[PC_COUNT];

// hardware counters of hw_perf.csv usable in HW / HYBRID mode
// (reference hw_perf_t, power_interface.cc:194-226; -accelwattch_hybrid_perfsim_<name>)
enum HwCounter : int {
  HW_L1_RH = 0, HW_L1_RM, HW_L1_WH, HW_L1_WM, HW_CC_ACC, HW_SHRD_ACC, HW_DRAM_RD, HW_DRAM_WR, HW_L2_RH, HW_L2_RM,
  HW_L2_WH, HW_L2_WM, HW_NOC, HW_PIPE_DUTY, HW_NUM_SM_IDLE, HW_CYCLES, HW_VOLTAGE, HW_COUNT
};
extern const char* const kHwCounterName[HW_COUNT];  // option suffixes (SHARED_ACC, DRAM_RD, ...)

struct PowerReport {
  double cmp[PC_COUNT] = {};
  double dynamic_w[PA_COUNT] = {};
  double dynamic = 0;
  double static_w = 0;
  double static_mem = 0;    // the part of static_w from the LDS / L1 / L2 "unit in use" terms
  double static_issue = 0;  // core static power weighted by issue (calibration column STATIC_ISSUEP)
  double constant = 0;
  double idle = 0;
  double total = 0;
  double uncapped = 0;      // the same activity at the nominal clock and voltage
  bool capped = false;      // the sample ran below the nominal clock (DVFS)
  double clock_ratio = 1.0;   // core clock / nominal of the sample
  double voltage_ratio = 1.0;
  std::string static_category;
};

class PowerModel {
 public:
  // mode: 0 SIM (simulated activity), 1 HW (activity from hw_perf.csv),
  // 2 HYBRID (hw for selected counters)
  bool load_xml(const std::string& path, std::string* err = nullptr);
  void set_param(const std::string& k, double v) { p_[k] = v; }
  double param(const std::string& k, double dflt = 0) const;
  // power of one sample whose activity was counted per core cycle, with the
  // core at `clock_ratio` x the nominal `core_mhz` (and the DVFS voltage)
  PowerReport compute(const Activity& act, double core_mhz, uint32_t n_sm, double clock_ratio = 1.0) const;
  // DVFS: V(s) / V(1), and the governor's clock ratio for the activity of the
  // last sample (1 without a power cap or when the nominal clock fits)
  double dvfs_voltage_ratio(double clock_ratio) const;
  double dvfs_clock_ratio(const Activity& act, double core_mhz, uint32_t n_sm) const;
  double dvfs_min_ratio() const;
  // activity of one kernel from stat deltas
  static Activity activity_from_stats(const std::vector<SMStats>& dsm, const std::vector<MemStats>& dmem,
                                      uint64_t cycles);
  // hw_perf.csv row -> activity (HW mode); returns false if not found
  static bool activity_from_hw_csv(const std::string& csv, const std::string& bench, const std::string& kernel,
                                   Activity& out, uint32_t n_sm);
  // HW (all counters from hardware) / HYBRID (counters with use_sim[i] set
  // come from the simulator) merge; instruction-side activity is always simulated
  static Activity merge_hw(const Activity& sim, const Activity& hw, const bool use_sim[HW_COUNT]);
  static double base_nj(int act);
  // per-access energies in use: the fixed table, or the architectural model's
  // (arch_energy.h, XML <param name="energy_model" value="1"/>)
  double base(int act) const { return (act >= 0 && act < PA_COUNT) ? base_[act] : 0.0; }
  void set_base(const double* e) {
    for (int i = 0; i < PA_COUNT; ++i) base_[i] = e[i];
  }
  PowerModel() {
    for (int i = 0; i < PA_COUNT; ++i) base_[i] = base_nj(i);
  }
  // coefficient vector (W per access per cycle at core_mhz)
  std::vector<double> coefficients(double core_mhz) const;
  // the sampler's coefficients at the nominal clock (engines' in-loop
  // sampling, power_eval.h)
  PwrCoef sampler_coef(double core_mhz) const;
  static Activity activity_of(const PwrSample& s);
  static PowerReport report_of(const PwrSample& s);

 private:
  std::map<std::string, double> p_;
  double base_[PA_COUNT];
};

// Per-kernel and cumulative avg / max / min of every component over the
// samples of a kernel (reference print_power_kernel_stats,
// gpgpu_sim_wrapper.cc:974-1041) and the optional per-sample trace.
class PowerTracker {
 public:
  void begin_kernel();
  void add_sample(const PowerReport& r, const Activity& a, uint64_t cycle);
  size_t kernel_samples() const { return k_n_; }
  // cycle-weighted mean core clock ratio of the kernel's samples (DVFS)
  double kernel_clock_ratio() const { return k_cyc_ > 0 ? k_clk_ / k_cyc_ : 1.0; }
  double kernel_avg_power() const { return k_n_ ? k_tot_.sum / (double)k_n_ : 0.0; }
  void write_kernel(std::ostream& os, const std::string& header) const;
  void write_trace_header(std::ostream& os) const;
  void write_trace_line(std::ostream& os, const PowerReport& r, uint64_t cycle) const;
  // steady-state levels: runs of >= n samples within +-dev% of their mean
  void set_steady(double dev_pct, uint32_t n) { st_dev_ = dev_pct; st_n_ = n; }
  void write_steady(std::ostream& os, const std::string& kernel) const;

 private:
  struct Agg {
    double sum = 0, mx = 0, mn = 0;
    bool any = false;
    void add(double v) {
      sum += v;
      mx = any ? (v > mx ? v : mx) : v;
      mn = any ? (v < mn ? v : mn) : v;
      any = true;
    }
  };
  Agg k_cmp_[PC_COUNT], k_act_[PA_COUNT], k_tot_, g_tot_;
  double k_lanes_ = 0;
  double k_clk_ = 0, k_cyc_ = 0;
  size_t k_n_ = 0, g_n_ = 0;
  std::vector<std::pair<uint64_t, double>> k_series_;
  double st_dev_ = 8;
  uint32_t st_n_ = 4;
};

}  // namespace asim
