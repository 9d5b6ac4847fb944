#include "power.h"

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <regex>
#include <sstream>

namespace asim {

const char* const kPwrActName[PA_COUNT] = {
    "TOT_INST", "FP_INT", "IC_H", "IC_M", "DC_RH", "DC_RM", "DC_WH", "DC_WM", "CC_H", "CC_M",
    "SHRD_ACC", "REG_RD", "REG_WR", "INT_ACC", "FP_ACC", "DP_ACC", "INT_MUL_ACC", "FP_MUL_ACC",
    "FP_SQRT_ACC", "FP_LG_ACC", "FP_SIN_ACC", "FP_EXP_ACC", "DP_MUL_ACC", "TENSOR_ACC", "TEX_ACC",
    "MEM_RD", "MEM_WR", "MEM_PRE", "L2_RH", "L2_RM", "L2_WH", "L2_WM", "NOC_A", "PIPE_A"};

const char* const kPwrCmpName[PC_COUNT] = {
    "IBP", "ICP", "DCP", "TCP", "CCP", "SHRDP", "RFP", "INTP", "FPUP", "DPUP", "INT_MUL24P", "INT_MUL32P", "INT_MULP",
    "INT_DIVP", "FP_MULP", "FP_DIVP", "FP_SQRTP", "FP_LGP", "FP_SINP", "FP_EXP", "DP_MULP", "DP_DIVP", "TENSORP", "TEXP",
    "SCHEDP", "L2CP", "MCP", "NOCP", "DRAMP", "PIPEP", "IDLE_COREP", "CONSTP", "STATICP"};

const char* const kHwCounterName[HW_COUNT] = {"L1_RH", "L1_RM", "L1_WH", "L1_WM", "CC_ACC", "SHARED_ACC",
                                              "DRAM_RD", "DRAM_WR", "L2_RH", "L2_RM", "L2_WH", "L2_WM",
                                              "NOC", "PIPE_DUTY", "NUM_SM_IDLE", "CYCLES", "VOLTAGE"};

// Per-access base energies (nJ) for a 12-16 nm class GPU.  These play the
// role of McPAT's per-access energies; the XML scaling factors calibrate
// them (util: accel_sim_framework_distributed_amd.power.calibrate).
double PowerModel::base_nj(int act) {
  static const double e[PA_COUNT] = {
      0.0100,  // TOT_INST   instruction buffer per warp instruction
      0.0250,  // FP_INT     scheduler per non-memory warp instruction
      0.0150,  // IC_H
      0.0500,  // IC_M
      0.0450,  // DC_RH      L1 read hit (per 128B access)
      0.0600,  // DC_RM
      0.0450,  // DC_WH
      0.0550,  // DC_WM
      0.0080,  // CC_H
      0.0300,  // CC_M
      0.0300,  // SHRD_ACC
      0.0040,  // REG_RD     per warp operand read
      0.0050,  // REG_WR
      0.0015,  // INT_ACC    per lane op
      0.0030,  // FP_ACC
      0.0080,  // DP_ACC
      0.0040,  // INT_MUL_ACC
      0.0040,  // FP_MUL_ACC
      0.0120,  // FP_SQRT_ACC
      0.0120,  // FP_LG_ACC
      0.0120,  // FP_SIN_ACC
      0.0120,  // FP_EXP_ACC
      0.0150,  // DP_MUL_ACC
      0.0600,  // TENSOR_ACC
      0.0400,  // TEX_ACC
      0.4000,  // MEM_RD     per 32B DRAM access
      0.4500,  // MEM_WR
      0.1000,  // MEM_PRE
      0.0600,  // L2_RH
      0.0800,  // L2_RM
      0.0600,  // L2_WH
      0.0800,  // L2_WM
      0.0250,  // NOC_A      per flit
      0.0050,  // PIPE_A
  };
  return (act >= 0 && act < PA_COUNT) ? e[act] : 0.0;
}

bool PowerModel::load_xml(const std::string& path, std::string* err) {
  std::ifstream f(path);
  if (!f) {
    if (err) *err = "cannot open " + path;
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  std::regex re("<param\\s+name\\s*=\\s*\"([^\"]+)\"\\s+value\\s*=\\s*\"([^\"]*)\"");
  for (auto it = std::sregex_iterator(s.begin(), s.end(), re); it != std::sregex_iterator(); ++it) {
    const std::string k = (*it)[1], v = (*it)[2];
    char* end = nullptr;
    double x = strtod(v.c_str(), &end);
    if (end != v.c_str()) p_[k] = x;
  }
  return true;
}

double PowerModel::param(const std::string& k, double dflt) const {
  auto it = p_.find(k);
  return it == p_.end() ? dflt : it->second;
}

std::vector<double> PowerModel::coefficients(double core_mhz) const {
  // W contributed by one access per core cycle
  std::vector<double> c(PA_COUNT);
  for (int i = 0; i < PA_COUNT; ++i) c[i] = base(i) * 1e-9 * param(kPwrActName[i], 1.0) * core_mhz * 1e6;
  return c;
}

PwrCoef PowerModel::sampler_coef(double core_mhz) const {
  PwrCoef k{};
  const auto c = coefficients(core_mhz);
  for (int i = 0; i < PA_COUNT; ++i) k.coef[i] = c[i];
  k.constant = param("constant_power", 0);
  k.idle_core = param("idle_core_power", 0);
  static const char* const cat[7] = {"light", "cat1", "cat2", "cat3", "cat4", "cat5", "cat6"};
  for (int i = 0; i < 7; ++i) {
    k.st_flane[i] = param(std::string("static_") + cat[i] + "_flane", 0);
    k.st_addlane[i] = param(std::string("static_") + cat[i] + "_addlane", 0);
  }
  k.st_shared = param("static_shared_flane", 0);
  k.st_l1 = param("static_l1_flane", 0);
  k.st_l2 = param("static_l2_flane", 0);
  k.st_issue_w = param("static_issue_weight", 0);
  return k;
}

Activity PowerModel::activity_of(const PwrSample& s) {
  Activity a;
  for (int i = 0; i < PA_COUNT; ++i) a.a[i] = s.act[i];
  a.cycles = s.cycles;
  a.idle_sms = s.idle_sms;
  a.avg_lanes = s.lanes;
  a.issue_frac = s.issue_frac;
  a.int_used = s.unit_mask & 1u;
  a.fp_used = s.unit_mask & 2u;
  a.dp_used = s.unit_mask & 4u;
  a.sfu_used = s.unit_mask & 8u;
  a.tex_used = s.unit_mask & 16u;
  a.tensor_used = s.unit_mask & 32u;
  return a;
}

PowerReport PowerModel::report_of(const PwrSample& o) {
  static const char* const cat[7] = {"light", "cat1", "cat2", "cat3", "cat4", "cat5", "cat6"};
  PowerReport r;
  for (int i = 0; i < PC_COUNT; ++i) r.cmp[i] = o.cmp[i];
  for (int i = 0; i < PA_COUNT; ++i) r.dynamic_w[i] = o.dyn[i];
  r.dynamic = o.dynamic;
  r.static_w = o.static_w;
  r.static_mem = o.static_mem;
  r.static_issue = o.static_issue;
  r.constant = o.constant;
  r.idle = o.idle;
  r.total = o.total;
  r.uncapped = o.total;
  r.static_category = cat[o.category < 7 ? o.category : 0];
  return r;
}

PowerReport PowerModel::compute(const Activity& a, double core_mhz, uint32_t n_sm, double clock_ratio) const {
  const double s = clock_ratio > 0 ? clock_ratio : 1.0;
  const double vr = s < 1.0 ? dvfs_voltage_ratio(s) : 1.0;
  const PwrCoef k = sampler_coef(core_mhz * s);
  // a.voltage: the HW-mode chip voltage ratio (hw_perf.csv); vr: DVFS
  const double v2 = a.voltage * a.voltage * vr * vr;
  PwrSample o{};
  for (int i = 0; i < PA_COUNT; ++i) o.act[i] = a.a[i];
  o.cycles = a.cycles;
  o.idle_sms = a.idle_sms;
  o.lanes = a.avg_lanes;
  o.issue_frac = a.issue_frac >= 0 ? a.issue_frac : (n_sm ? std::max(0.0, 1.0 - a.idle_sms / n_sm) : 1.0);
  o.unit_mask = (a.int_used ? 1u : 0u) | (a.fp_used ? 2u : 0u) | (a.dp_used ? 4u : 0u) | (a.sfu_used ? 8u : 0u) |
                (a.tex_used ? 16u : 0u) | (a.tensor_used ? 32u : 0u);
  pwr_power(k, k.coef, n_sm, v2, a.voltage * a.voltage, vr, o);
  PowerReport r = report_of(o);
  r.clock_ratio = s;
  r.voltage_ratio = vr;
  r.capped = s < 1.0;
  r.uncapped = s < 1.0 ? compute(a, core_mhz, n_sm, 1.0).total : r.total;
  return r;
}

double PowerModel::dvfs_voltage_ratio(double s) const {
  const double vf = param("dvfs_v_floor", 0.6);
  return vf + (1.0 - vf) * s;
}

double PowerModel::dvfs_min_ratio() const {
  return std::min(1.0, std::max(0.05, param("dvfs_min_clock_ratio", 0.5)));
}

double PowerModel::dvfs_clock_ratio(const Activity& a, double core_mhz, uint32_t n_sm) const {
  const double cap = param("power_cap", 0);
  if (cap <= 0 || compute(a, core_mhz, n_sm, 1.0).total <= cap) return 1.0;
  // P(s) rises monotonically with s: bisect for the highest s under the cap
  double lo = dvfs_min_ratio(), hi = 1.0;
  if (compute(a, core_mhz, n_sm, lo).total >= cap) return lo;
  for (int i = 0; i < 40; ++i) {
    const double m = 0.5 * (lo + hi);
    (compute(a, core_mhz, n_sm, m).total <= cap ? lo : hi) = m;
  }
  return lo;
}

Activity PowerModel::merge_hw(const Activity& sim, const Activity& hw, const bool use_sim[HW_COUNT]) {
  Activity a = sim;
  auto pick = [&](int hwc, int act) {
    if (!use_sim[hwc]) a.a[act] = hw.a[act];
  };
  pick(HW_L1_RH, PA_DC_RH);
  pick(HW_L1_RM, PA_DC_RM);
  pick(HW_L1_WH, PA_DC_WH);
  pick(HW_L1_WM, PA_DC_WM);
  pick(HW_CC_ACC, PA_CC_H);
  pick(HW_SHRD_ACC, PA_SHRD_ACC);
  pick(HW_DRAM_RD, PA_MEM_RD);
  pick(HW_DRAM_WR, PA_MEM_WR);
  pick(HW_L2_RH, PA_L2_RH);
  pick(HW_L2_RM, PA_L2_RM);
  pick(HW_L2_WH, PA_L2_WH);
  pick(HW_L2_WM, PA_L2_WM);
  pick(HW_NOC, PA_NOC_A);
  pick(HW_PIPE_DUTY, PA_PIPE_A);
  if (!use_sim[HW_NUM_SM_IDLE]) a.idle_sms = hw.idle_sms;
  if (!use_sim[HW_VOLTAGE]) a.voltage = hw.voltage;
  if (!use_sim[HW_CYCLES] && hw.cycles > 0) {
    // the simulated instruction-side counts stay; the sample spans the HW time
    a.cycles = hw.cycles;
  }
  return a;
}

void PowerTracker::begin_kernel() {
  for (auto& x : k_cmp_) x = Agg{};
  for (auto& x : k_act_) x = Agg{};
  k_tot_ = Agg{};
  k_lanes_ = 0;
  k_clk_ = k_cyc_ = 0;
  k_n_ = 0;
  k_series_.clear();
}

void PowerTracker::add_sample(const PowerReport& r, const Activity& a, uint64_t cycle) {
  for (int i = 0; i < PC_COUNT; ++i) k_cmp_[i].add(r.cmp[i]);
  for (int i = 0; i < PA_COUNT; ++i) k_act_[i].add(a.a[i]);
  k_tot_.add(r.total);
  g_tot_.add(r.total);
  k_lanes_ += a.avg_lanes;
  k_clk_ += r.clock_ratio * a.cycles;
  k_cyc_ += a.cycles;
  ++k_n_;
  ++g_n_;
  k_series_.emplace_back(cycle, r.total);
}

void PowerTracker::write_kernel(std::ostream& os, const std::string& header) const {
  const double n = k_n_ ? (double)k_n_ : 1.0;
  os << header << "\n";
  os << "Kernel Average Power Data:\n";
  os << "kernel_avg_power = " << k_tot_.sum / n << "\n";
  for (int i = 0; i < PC_COUNT; ++i) os << "gpu_avg_" << kPwrCmpName[i] << " = " << k_cmp_[i].sum / n << "\n";
  for (int i = 0; i < PA_COUNT; ++i) os << "gpu_avg_" << kPwrActName[i] << " = " << k_act_[i].sum / n << "\n";
  os << "gpu_avg_threads_per_warp = " << k_lanes_ / n << "\n";
  os << "kernel_avg_clock_ratio = " << kernel_clock_ratio() << "\n";
  for (int i = 0; i < PA_COUNT; ++i) os << "gpu_tot_" << kPwrActName[i] << " = " << k_act_[i].sum << "\n";
  os << "\nKernel Maximum Power Data:\n";
  os << "kernel_max_power = " << k_tot_.mx << "\n";
  for (int i = 0; i < PC_COUNT; ++i) os << "gpu_max_" << kPwrCmpName[i] << " = " << k_cmp_[i].mx << "\n";
  for (int i = 0; i < PA_COUNT; ++i) os << "gpu_max_" << kPwrActName[i] << " = " << k_act_[i].mx << "\n";
  os << "\nKernel Minimum Power Data:\n";
  os << "kernel_min_power = " << k_tot_.mn << "\n";
  for (int i = 0; i < PC_COUNT; ++i) os << "gpu_min_" << kPwrCmpName[i] << " = " << k_cmp_[i].mn << "\n";
  for (int i = 0; i < PA_COUNT; ++i) os << "gpu_min_" << kPwrActName[i] << " = " << k_act_[i].mn << "\n";
  os << "\nAccumulative Power Statistics Over Previous Kernels:\n";
  os << "gpu_tot_avg_power = " << (g_n_ ? g_tot_.sum / (double)g_n_ : 0.0) << "\n";
  os << "gpu_tot_max_power = " << g_tot_.mx << "\n";
  os << "gpu_tot_min_power = " << g_tot_.mn << "\n\n\n";
  os.flush();
}

void PowerTracker::write_trace_header(std::ostream& os) const {
  os << "cycle,total_power";
  for (int i = 0; i < PC_COUNT; ++i) os << "," << kPwrCmpName[i];
  // the memory-unit share of STATICP (calibration splits the static factor),
  // and the core static power weighted by issue (the calibration's
  // alternative column, csrc/power/power_eval.h pwr_power)
  os << ",STATIC_MEMP,STATIC_ISSUEP\n";
}

void PowerTracker::write_trace_line(std::ostream& os, const PowerReport& r, uint64_t cycle) const {
  os << cycle << "," << r.total;
  for (int i = 0; i < PC_COUNT; ++i) os << "," << r.cmp[i];
  os << "," << r.static_mem << "," << r.static_issue << "\n";
}

void PowerTracker::write_steady(std::ostream& os, const std::string& kernel) const {
  // greedy left-to-right segmentation of the sample series
  size_t i = 0;
  while (i < k_series_.size()) {
    size_t j = i + 1;
    double sum = k_series_[i].second;
    while (j < k_series_.size()) {
      const double mean = (sum + k_series_[j].second) / (double)(j - i + 1);
      bool ok = true;
      for (size_t q = i; q <= j && ok; ++q)
        ok = std::fabs(k_series_[q].second - mean) <= mean * st_dev_ / 100.0;
      if (!ok) break;
      sum += k_series_[j].second;
      ++j;
    }
    if (j - i >= st_n_)
      os << kernel << "," << k_series_[i].first << "," << k_series_[j - 1].first << "," << (j - i) << ","
         << sum / (double)(j - i) << "\n";
    i = j;
  }
}

// the sums of a statistics image (power_eval.h step 2, host loops)
void pwr_sums(const std::vector<SMStats>& sm, const std::vector<MemStats>& mem, double* S) {
  for (int j = 0; j < PS_COUNT; ++j) S[j] = 0;
  for (const auto& s : sm)
    for (int r = 0; r < PR_COUNT; ++r) {
      const int j = pwr_sum_of(r);
      if (j >= 0) S[j] += (double)pwr_raw_sm(s, r);
    }
  for (const auto& m : mem)
    for (int r = 0; r < PR_COUNT; ++r) {
      const int j = pwr_sum_of(r);
      if (j >= 0) S[j] += (double)pwr_raw_mem(m, r);
    }
}

Activity PowerModel::activity_from_stats(const std::vector<SMStats>& dsm, const std::vector<MemStats>& dmem,
                                         uint64_t cycles) {
  double S[PS_COUNT];
  pwr_sums(dsm, dmem, S);
  PwrSample o{};
  pwr_activity(S, (double)cycles, (uint32_t)dsm.size(), o);
  return activity_of(o);
}

bool PowerModel::activity_from_hw_csv(const std::string& csv, const std::string& bench, const std::string& kernel,
                                      Activity& out, uint32_t n_sm) {
  std::ifstream f(csv);
  if (!f) return false;
  std::string line;
  std::getline(f, line);
  std::vector<std::string> hdr;
  {
    std::stringstream ss(line);
    std::string t;
    while (std::getline(ss, t, ',')) hdr.push_back(t);
  }
  while (std::getline(f, line)) {
    std::vector<std::string> v;
    std::stringstream ss(line);
    std::string t;
    while (std::getline(ss, t, ',')) v.push_back(t);
    if (v.size() < 2 || v[0] != bench || v[1] != kernel) continue;
    Activity a;
    auto get = [&](const char* name) -> double {
      for (size_t i = 0; i < hdr.size() && i < v.size(); ++i)
        if (hdr[i] == name) return atof(v[i].c_str());
      return 0;
    };
    a.a[PA_DC_RH] = get("L1_RH");
    a.a[PA_DC_RM] = get("L1_RM");
    a.a[PA_DC_WH] = get("L1_WH");
    a.a[PA_DC_WM] = get("L1_WM");
    a.a[PA_CC_H] = get("CC_ACC");
    a.a[PA_SHRD_ACC] = get("SHRD_ACC");
    a.a[PA_MEM_RD] = get("DRAM_Rd");
    a.a[PA_MEM_WR] = get("DRAM_Wr");
    a.a[PA_L2_RH] = get("L2_RH");
    a.a[PA_L2_RM] = get("L2_RM");
    a.a[PA_L2_WH] = get("L2_WH");
    a.a[PA_L2_WM] = get("L2_WM");
    a.a[PA_NOC_A] = get("NOC");
    a.cycles = get("Elapsed_Cycles");
    a.idle_sms = get("Num_Idle_SMs");
    a.voltage = get("Chip Voltage") > 0 ? get("Chip Voltage") : 1.0;
    double duty = get("Pipeline_Duty");
    a.a[PA_PIPE_A] = duty * a.cycles * (n_sm - a.idle_sms);
    a.int_used = true;
    a.fp_used = true;
    a.avg_lanes = 32;
    out = a;
    return true;
  }
  return false;
}

}  // namespace asim
