// Power sample evaluation shared by the host model (power.cc), the CPU engine
// and the GPU engine's in-kernel sampler (engine_kernel): one implementation,
// compiled for host and device, so a sample is bit-identical wherever it is
// computed (floating-point contraction is off in this header: the device
// compiler would otherwise fuse a*b+c into FMAs the host does not use).
//
// A sample in three steps:
//  1. raw counters: one row of PR_COUNT integers per unit (SM or memory
//     channel), cumulative statistics read from the unit's state;
//  2. sums: S = rows x M, M the 0/1 map of raw counters onto the model's
//     inputs (pwr_sum_of), summed over all units.  Every partial sum is an
//     integer below 2^53, so the result is exact in any order: the GPU engine
//     evaluates it as f64 MFMA tiles (units x raw counters by raw counters x
//     sums), the host as plain loops;
//  3. the sample: deltas of S since the previous sample -> activity per core
//     cycle -> per-activity dynamic power, static / idle / constant power
//     (reference power_interface.cc:52-188 mcpat_cycle, gpgpu_sim_wrapper.cc
//     calculate_static_power / update_components_power).
#pragma once
#include <cstdint>

#include "../model/hd.h"
#include "../model/mem.h"
#include "../model/sm.h"

// no fused multiply-add in the functions below (scoped to each body)
#if defined(__clang__)
#define PWR_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define PWR_NO_CONTRACT
#endif

namespace asim {

enum PwrAct : int {
  PA_TOT_INST = 0, PA_FP_INT, PA_IC_H, PA_IC_M, PA_DC_RH, PA_DC_RM, PA_DC_WH, PA_DC_WM, PA_CC_H, PA_CC_M,
  PA_SHRD_ACC, PA_REG_RD, PA_REG_WR, PA_INT_ACC, PA_FP_ACC, PA_DP_ACC, PA_INT_MUL_ACC, PA_FP_MUL_ACC,
  PA_FP_SQRT_ACC, PA_FP_LG_ACC, PA_FP_SIN_ACC, PA_FP_EXP_ACC, PA_DP_MUL_ACC, PA_TENSOR_ACC, PA_TEX_ACC,
  PA_MEM_RD, PA_MEM_WR, PA_MEM_PRE, PA_L2_RH, PA_L2_RM, PA_L2_WH, PA_L2_WM, PA_NOC_A, PA_PIPE_A, PA_COUNT
};

// report components (labels of the reference's pwr_cmp_t,
// accelwattch/gpgpu_sim_wrapper.cc:42-77)
enum PwrCmp : int {
  PC_IB = 0, PC_IC, PC_DC, PC_TC, PC_CC, PC_SHRD, PC_RF, PC_INT, PC_FPU, PC_DPU, PC_INT_MUL24, PC_INT_MUL32, PC_INT_MUL,
  PC_INT_DIV, PC_FP_MUL, PC_FP_DIV, PC_FP_SQRT, PC_FP_LG, PC_FP_SIN, PC_FP_EXP, PC_DP_MUL, PC_DP_DIV, PC_TENSOR, PC_TEX,
  PC_SCHED, PC_L2C, PC_MC, PC_NOC, PC_DRAM, PC_PIPE, PC_IDLE_CORE, PC_CONST, PC_STATIC, PC_COUNT
};

// activity -> report component
SIM_HDI int pwr_cmp_of(int act) {
  switch (act) {
    case PA_TOT_INST: return PC_IB;
    case PA_FP_INT: return PC_SCHED;
    case PA_IC_H: case PA_IC_M: return PC_IC;
    case PA_DC_RH: case PA_DC_RM: case PA_DC_WH: case PA_DC_WM: return PC_DC;
    case PA_CC_H: case PA_CC_M: return PC_CC;
    case PA_SHRD_ACC: return PC_SHRD;
    case PA_REG_RD: case PA_REG_WR: return PC_RF;
    case PA_INT_ACC: return PC_INT;
    case PA_FP_ACC: return PC_FPU;
    case PA_DP_ACC: return PC_DPU;
    case PA_INT_MUL_ACC: return PC_INT_MUL;
    case PA_FP_MUL_ACC: return PC_FP_MUL;
    case PA_FP_SQRT_ACC: return PC_FP_SQRT;
    case PA_FP_LG_ACC: return PC_FP_LG;
    case PA_FP_SIN_ACC: return PC_FP_SIN;
    case PA_FP_EXP_ACC: return PC_FP_EXP;
    case PA_DP_MUL_ACC: return PC_DP_MUL;
    case PA_TENSOR_ACC: return PC_TENSOR;
    case PA_TEX_ACC: return PC_TEX;
    case PA_MEM_RD: case PA_MEM_WR: return PC_DRAM;
    case PA_MEM_PRE: return PC_MC;
    case PA_L2_RH: case PA_L2_RM: case PA_L2_WH: case PA_L2_WM: return PC_L2C;
    case PA_NOC_A: return PC_NOC;
    default: return PC_PIPE;
  }
}

// ---- raw counters of one unit's row ----------------------------------------
enum PwrRaw : int {
  PR_WARP = 0, PR_THREAD, PR_MEMI, PR_ACTIVE,
  PR_L1_GR_HIT, PR_L1_LR_HIT, PR_L1_GR_MISS, PR_L1_LR_MISS, PR_L1_GR_MSHR, PR_L1_LR_MSHR, PR_L1_GR_BYP,
  PR_L1_GW_MISS, PR_L1_LW_MISS, PR_L1_GW_BYP, PR_L1_AT_BYP, PR_L1_GW_HIT, PR_L1_LW_HIT,
  PR_CONST, PR_SHMEM, PR_RF_RD, PR_RF_WR, PR_PKT_OUT, PR_PKT_IN,
  PR_KIND0,  // + PWR_INT - 1 .. PWR_SALU - 1: issued lanes per unit kind
  PR_DRAM_RD = PR_KIND0 + (PWR_KINDS - 1), PR_DRAM_WR, PR_DRAM_PRE,
  PR_L2_RD_HIT, PR_L2_AT_HIT, PR_L2_RD_MISS, PR_L2_RD_MSHR, PR_L2_AT_MISS, PR_L2_WR_HIT, PR_L2_WR_MISS,
  PR_BUSY,  // SM cycles with an instruction issued
  PR_COUNT
};
constexpr int kPwrRawPad = (PR_COUNT + 3) / 4 * 4;  // k-steps of 4 (f64 MFMA 16x16x4)

// ---- sums (model inputs) ----------------------------------------------------
enum PwrSum : int {
  PS_WARP = 0, PS_THREAD, PS_MEMI, PS_ACTIVE, PS_DC_RH, PS_DC_RM, PS_DC_WM, PS_DC_WH, PS_CC, PS_SHRD, PS_RF_RD,
  PS_RF_WR, PS_NOC,
  PS_KIND0,  // + kind - 1
  PS_DRAM_RD = PS_KIND0 + (PWR_KINDS - 1), PS_DRAM_WR, PS_DRAM_PRE, PS_L2_RH, PS_L2_RM, PS_L2_WH, PS_L2_WM,
  PS_BUSY,
  PS_COUNT
};
constexpr int kPwrSumPad = (PS_COUNT + 15) / 16 * 16;  // column tiles of 16

// the 0/1 map M: raw counter -> the sum it adds to (-1: none)
SIM_HDI int pwr_sum_of(int r) {
  if (r >= PR_KIND0 && r < PR_KIND0 + PWR_KINDS - 1) return PS_KIND0 + (r - PR_KIND0);
  switch (r) {
    case PR_WARP: return PS_WARP;
    case PR_THREAD: return PS_THREAD;
    case PR_MEMI: return PS_MEMI;
    case PR_ACTIVE: return PS_ACTIVE;
    case PR_L1_GR_HIT: case PR_L1_LR_HIT: return PS_DC_RH;
    case PR_L1_GR_MISS: case PR_L1_LR_MISS: case PR_L1_GR_MSHR: case PR_L1_LR_MSHR: case PR_L1_GR_BYP: return PS_DC_RM;
    case PR_L1_GW_MISS: case PR_L1_LW_MISS: case PR_L1_GW_BYP: case PR_L1_AT_BYP: return PS_DC_WM;
    case PR_L1_GW_HIT: case PR_L1_LW_HIT: return PS_DC_WH;
    case PR_CONST: return PS_CC;
    case PR_SHMEM: return PS_SHRD;
    case PR_RF_RD: return PS_RF_RD;
    case PR_RF_WR: return PS_RF_WR;
    case PR_PKT_OUT: case PR_PKT_IN: return PS_NOC;
    case PR_DRAM_RD: return PS_DRAM_RD;
    case PR_DRAM_WR: return PS_DRAM_WR;
    case PR_DRAM_PRE: return PS_DRAM_PRE;
    case PR_L2_RD_HIT: case PR_L2_AT_HIT: return PS_L2_RH;
    case PR_L2_RD_MISS: case PR_L2_RD_MSHR: case PR_L2_AT_MISS: return PS_L2_RM;
    case PR_L2_WR_HIT: return PS_L2_WH;
    case PR_L2_WR_MISS: return PS_L2_WM;
    case PR_BUSY: return PS_BUSY;
    default: return -1;
  }
}

// raw counter r of an SM / of a memory sub-partition's statistics (0 where
// the unit has no such counter)
SIM_HDI uint64_t pwr_raw_sm(const SMStats& s, int r) {
  if (r >= PR_KIND0 && r < PR_KIND0 + PWR_KINDS - 1) return s.power_acc[1 + (r - PR_KIND0)];
  switch (r) {
    case PR_WARP: return s.warp_insn;
    case PR_THREAD: return s.thread_insn;
    case PR_MEMI: return s.mem_insn;
    case PR_ACTIVE: return s.active_cycles;
    case PR_BUSY: return s.busy_cycles;
    case PR_L1_GR_HIT: return s.l1[L1T_GLOBAL_R][L1O_HIT];
    case PR_L1_LR_HIT: return s.l1[L1T_LOCAL_R][L1O_HIT];
    case PR_L1_GR_MISS: return s.l1[L1T_GLOBAL_R][L1O_MISS];
    case PR_L1_LR_MISS: return s.l1[L1T_LOCAL_R][L1O_MISS];
    case PR_L1_GR_MSHR: return s.l1[L1T_GLOBAL_R][L1O_MSHR_HIT];
    case PR_L1_LR_MSHR: return s.l1[L1T_LOCAL_R][L1O_MSHR_HIT];
    case PR_L1_GR_BYP: return s.l1[L1T_GLOBAL_R][L1O_BYPASS];
    case PR_L1_GW_MISS: return s.l1[L1T_GLOBAL_W][L1O_MISS];
    case PR_L1_LW_MISS: return s.l1[L1T_LOCAL_W][L1O_MISS];
    case PR_L1_GW_BYP: return s.l1[L1T_GLOBAL_W][L1O_BYPASS];
    case PR_L1_AT_BYP: return s.l1[L1T_ATOMIC][L1O_BYPASS];
    case PR_L1_GW_HIT: return s.l1[L1T_GLOBAL_W][L1O_HIT];
    case PR_L1_LW_HIT: return s.l1[L1T_LOCAL_W][L1O_HIT];
    case PR_CONST: return s.power_acc[PWR_CONST_OPERAND];
    case PR_SHMEM: return s.shmem_acc;
    case PR_RF_RD: return s.rf_reads;
    case PR_RF_WR: return s.rf_writes;
    case PR_PKT_OUT: return s.pkts_out;
    case PR_PKT_IN: return s.pkts_in;
    default: return 0;
  }
}
SIM_HDI uint64_t pwr_raw_mem(const MemStats& m, int r) {
  switch (r) {
    case PR_DRAM_RD: return m.dram_rd;
    case PR_DRAM_WR: return m.dram_wr;
    case PR_DRAM_PRE: return m.dram_pre;
    case PR_L2_RD_HIT: return m.l2[L2T_RD][L2O_HIT];
    case PR_L2_AT_HIT: return m.l2[L2T_ATOM][L2O_HIT];
    case PR_L2_RD_MISS: return m.l2[L2T_RD][L2O_MISS];
    case PR_L2_RD_MSHR: return m.l2[L2T_RD][L2O_MSHR_HIT];
    case PR_L2_AT_MISS: return m.l2[L2T_ATOM][L2O_MISS];
    case PR_L2_WR_HIT: return m.l2[L2T_WR][L2O_HIT];
    case PR_L2_WR_MISS: return m.l2[L2T_WR][L2O_MISS];
    default: return 0;
  }
}

// per-simulation coefficients (host-prepared from the AccelWattch XML and the
// nominal core clock; power.cc PowerModel::sampler_coef)
struct PwrCoef {
  double coef[PA_COUNT];  // W contributed by one access per core cycle
  double constant;
  double idle_core;
  double st_flane[7], st_addlane[7];  // static categories: light, cat1 .. cat6
  double st_shared, st_l1, st_l2;
  // share of the core static power that follows instruction issue instead of
  // residency (XML static_issue_weight; 0 = the reference's categorical
  // static power of every SM with a live warp)
  double st_issue_w;
};

// one power sample: the activity of the sample and its power
struct PwrSample {
  uint64_t now;  // core cycle at the end of the sample
  double cycles;
  double idle_sms;
  double lanes;  // active threads per warp instruction
  double issue_frac;  // SM-cycles with an instruction issued / (SMs x cycles)
  double act[PA_COUNT];
  double dyn[PA_COUNT];
  double cmp[PC_COUNT];
  double dynamic, static_w, static_mem, constant, idle, total;
  double static_issue;  // the core static power weighted by issue instead of residency (calibration column)
  uint32_t category;  // 0 light, 1..6 cat1..cat6
  uint32_t unit_mask;  // bit 0 int, 1 fp, 2 dp, 3 sfu, 4 tex, 5 tensor
};

// step 3a: activity of a sample from the deltas of the sums
SIM_HDI void pwr_activity(const double* d, double cycles, uint32_t n_sm, PwrSample& o) {
  PWR_NO_CONTRACT
  for (int i = 0; i < PA_COUNT; ++i) o.act[i] = 0;
  o.cycles = cycles;
  const double warp = d[PS_WARP], thread = d[PS_THREAD];
  o.lanes = warp > 0 ? thread / warp : 0;
  o.act[PA_TOT_INST] = warp;
  o.act[PA_FP_INT] = warp - d[PS_MEMI];
  o.act[PA_IC_H] = warp;
  o.act[PA_DC_RH] = d[PS_DC_RH];
  o.act[PA_DC_RM] = d[PS_DC_RM];
  o.act[PA_DC_WH] = d[PS_DC_WH];
  o.act[PA_DC_WM] = d[PS_DC_WM];
  o.act[PA_CC_H] = d[PS_CC];
  o.act[PA_SHRD_ACC] = d[PS_SHRD];
  o.act[PA_REG_RD] = d[PS_RF_RD];
  o.act[PA_REG_WR] = d[PS_RF_WR];
  o.act[PA_NOC_A] = d[PS_NOC];
  // lanes charged at issue per unit kind (incexecstat)
  const double* k = d + PS_KIND0 - 1;  // k[PWR_x]
  o.act[PA_INT_ACC] = k[PWR_INT] + k[PWR_SALU];
  o.act[PA_INT_MUL_ACC] = k[PWR_INT_MUL];
  o.act[PA_FP_ACC] = k[PWR_FP];
  o.act[PA_FP_MUL_ACC] = k[PWR_FP_MUL];
  o.act[PA_DP_ACC] = k[PWR_DP];
  o.act[PA_DP_MUL_ACC] = k[PWR_DP_MUL];
  o.act[PA_FP_SQRT_ACC] = k[PWR_SQRT];
  o.act[PA_FP_LG_ACC] = k[PWR_LG];
  o.act[PA_FP_SIN_ACC] = k[PWR_SIN];
  o.act[PA_FP_EXP_ACC] = k[PWR_EXP];
  o.act[PA_TENSOR_ACC] = k[PWR_TENSOR];
  o.act[PA_TEX_ACC] = k[PWR_TEX];
  o.act[PA_PIPE_A] = warp;
  o.act[PA_MEM_RD] = d[PS_DRAM_RD];
  o.act[PA_MEM_WR] = d[PS_DRAM_WR];
  o.act[PA_MEM_PRE] = d[PS_DRAM_PRE];
  o.act[PA_L2_RH] = d[PS_L2_RH];
  o.act[PA_L2_RM] = d[PS_L2_RM];
  o.act[PA_L2_WH] = d[PS_L2_WH];
  o.act[PA_L2_WM] = d[PS_L2_WM];
  uint32_t um = 0;
  if (k[PWR_INT] + k[PWR_INT_MUL] + k[PWR_SALU] > 0) um |= 1u;
  if (k[PWR_FP] + k[PWR_FP_MUL] > 0) um |= 2u;
  if (k[PWR_DP] + k[PWR_DP_MUL] > 0) um |= 4u;
  if (k[PWR_SQRT] + k[PWR_LG] + k[PWR_SIN] + k[PWR_EXP] > 0) um |= 8u;
  if (k[PWR_TEX] > 0) um |= 16u;
  if (k[PWR_TENSOR] > 0) um |= 32u;
  o.unit_mask = um;
  double idle = cycles > 0 ? (double)n_sm - d[PS_ACTIVE] / cycles : 0;
  o.idle_sms = idle < 0 ? 0 : idle;
  const double iss = (cycles > 0 && n_sm) ? d[PS_BUSY] / cycles / (double)n_sm : 0;
  o.issue_frac = iss > 1 ? 1 : iss;
}

// step 3b: power of the sample.  `coef` is scaled for the sample's core clock;
// v2: core-rail dynamic voltage factor, vmem2: the HBM rail's, vr: static
// voltage ratio (1 / 1 / 1 at the nominal clock).  Same arithmetic, in the
// same order, as the reference's linear AccelWattch evaluation.
SIM_HDI void pwr_power(const PwrCoef& k, const double* coef, uint32_t n_sm, double v2, double vmem2, double vr,
                       PwrSample& o) {
  PWR_NO_CONTRACT
  const double cyc = o.cycles > 0 ? o.cycles : 1;
  o.dynamic = 0;
  for (int i = 0; i < PC_COUNT; ++i) o.cmp[i] = 0;
  for (int i = 0; i < PA_COUNT; ++i) {
    const bool dram = i == PA_MEM_RD || i == PA_MEM_WR || i == PA_MEM_PRE;  // the HBM rail keeps its voltage
    o.dyn[i] = coef[i] * (o.act[i] / cyc) * (dram ? vmem2 : v2);
    o.dynamic += o.dyn[i];
  }
  o.constant = k.constant;
  o.idle = k.idle_core * o.idle_sms * vr;
  // categorical static power by active unit mix (reference
  // calculate_static_power, gpgpu_sim_wrapper.cc:746-846)
  const uint32_t um = o.unit_mask;
  const uint32_t cat = (um & 32u) ? 6u : (um & 16u) ? 5u : (um & 8u) ? 4u : (um & 4u) ? 3u : (um & 2u) ? 2u
                     : (um & 1u) ? 1u : 0u;
  o.category = cat;
  const double lanes = o.lanes > 1 ? o.lanes : 1;
  const double busy_frac = n_sm ? (1.0 - o.idle_sms / n_sm > 0.0 ? 1.0 - o.idle_sms / n_sm : 0.0) : 1.0;
  const double st_base = k.st_flane[cat] + k.st_addlane[cat] * (lanes - 1);
  const double w = k.st_issue_w;
  double st = st_base * ((1.0 - w) * busy_frac + w * o.issue_frac);
  double smem = 0;
  if (o.act[PA_SHRD_ACC] > 0) smem += k.st_shared * busy_frac;
  if (o.act[PA_DC_RH] + o.act[PA_DC_RM] + o.act[PA_DC_WH] + o.act[PA_DC_WM] > 0) smem += k.st_l1 * busy_frac;
  if (o.act[PA_L2_RH] + o.act[PA_L2_RM] + o.act[PA_L2_WH] + o.act[PA_L2_WM] > 0) smem += k.st_l2;
  o.static_w = (st + smem) * vr;
  o.static_mem = smem * vr;
  o.static_issue = st_base * o.issue_frac * vr;
  o.total = o.dynamic + o.static_w + o.constant + o.idle;
  for (int i = 0; i < PA_COUNT; ++i) o.cmp[pwr_cmp_of(i)] += o.dyn[i];
  o.cmp[PC_IDLE_CORE] = o.idle;
  o.cmp[PC_CONST] = o.constant;
  o.cmp[PC_STATIC] = o.static_w;
}

}  // namespace asim
