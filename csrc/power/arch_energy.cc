#include "arch_energy.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <sstream>

namespace asim {

namespace {

// tabulated high-performance nodes: feature size (nm), nominal Vdd, gate and
// wire capacitance per um, leakage per um of width, 6T SRAM cell area (um^2,
// published bit cells: FinFET cells stop scaling as F^2)
struct Node {
  double nm, vdd, c_gate, c_wire, i_leak, cell;
};
constexpr Node kNodes[] = {
    {45, 1.00, 1.00, 0.20, 100, 0.346}, {32, 0.90, 0.95, 0.19, 110, 0.171}, {22, 0.85, 0.90, 0.18, 120, 0.092},
    {16, 0.80, 0.86, 0.18, 60, 0.074},  {12, 0.80, 0.85, 0.18, 60, 0.060}, {7, 0.75, 0.80, 0.19, 50, 0.027},
    {5, 0.72, 0.78, 0.20, 45, 0.021},   {3, 0.70, 0.75, 0.21, 40, 0.0199},
};

constexpr double kFemto = 1e-15, kNano = 1e-9;

// one gate-equivalent's switched energy (J): ~3 fF with its local wiring at
// 45 nm, scaled by feature size
double e_gate(const TechParams& t) { return 3.0 * kFemto * (t.node_nm / 45.0) * t.vdd * t.vdd; }

// 45 nm / 0.9 V reference energies of datapath operations (pJ, per lane):
// 32-bit integer add / multiply, fp32 add / multiply, fp64 add / multiply,
// a transcendental (quadratic interpolation + table), a 16-bit MAC
constexpr double kIntAdd = 0.1, kIntMul = 3.1, kFpAdd = 0.9, kFpMul = 3.7, kDpAdd = 2.2, kDpMul = 12.0,
                 kSfu = 10.0, kMac16 = 1.5;
double op_nj(double pj45, const TechParams& t) {
  return pj45 * 1e-3 * (t.node_nm / 45.0) * (t.vdd * t.vdd) / (0.9 * 0.9);
}

int ilog2(double v) { return v <= 1 ? 0 : (int)std::ceil(std::log2(v)); }

struct SubEval {
  double e_read, e_write, t, area_um2, leak_w;
  uint32_t rows, cols;
};

// one organisation of a logical array of `rows_total` x `cols_total` bits
// split into ndbl x ndwl subarrays; `read_cols` bits are sensed per access
SubEval eval_org(const TechParams& t, double rows_total, double cols_total, uint32_t ndwl, uint32_t ndbl,
                 double sensed_bits, double io_bits, double written_bits) {
  const double F = t.node_nm * 1e-3;  // um
  const double cell_w = std::sqrt(2.0 * t.sram_cell_um2), cell_h = std::sqrt(t.sram_cell_um2 / 2.0);
  const double R = rows_total / ndbl, C = cols_total / ndwl;
  // per-cell loads on the bitline (access drain + wire) and wordline (two gates + wire)
  const double c_bl_cell = 0.5 * t.c_gate * 1.5 * F + t.c_wire * cell_h;
  const double c_wl_cell = 2.0 * t.c_gate * 1.5 * F + t.c_wire * cell_w;
  const double c_bl = R * c_bl_cell * kFemto, c_wl = C * c_wl_cell * kFemto;
  const double vsw = 0.1 * t.vdd;  // read bitline swing (sense amplified)
  const double v2 = t.vdd * t.vdd;
  // activated: one row of subarrays along the wordline (ndwl of them)
  const double e_wl = ndwl * c_wl * v2;
  const double e_bl_rd = ndwl * C * c_bl * t.vdd * vsw;
  const double e_sa = sensed_bits * 4.0 * e_gate(t);
  // decoder + per activated subarray its wordline drivers, precharge and
  // column-mux control (the peripheral cost that bounds how finely an array
  // is worth dividing)
  const double e_dec = (ilog2(rows_total) + ilog2((double)ndwl * ndbl)) * 12.0 * e_gate(t) + ndwl * 40.0 * e_gate(t);
  // H-tree: from the array's centre to the activated subarrays and back
  // + peripheral strips: sense amplifiers / column mux below, decoder / drivers beside
  const double sub_w = C * cell_w + 12.0 * cell_w, sub_h = R * cell_h + 24.0 * cell_h;
  const double area = ndwl * ndbl * sub_w * sub_h;
  const double L = 0.5 * (std::sqrt(area) + ndwl * sub_w * 0.5);
  const double e_ht = (io_bits + ilog2(rows_total * ndwl)) * L * t.c_wire * kFemto * v2 * 0.5;
  SubEval r;
  r.e_read = e_wl + e_bl_rd + e_sa + e_dec + e_ht;
  // a write swings the written columns fully; the half-selected rest like a read
  const double wbits = std::min(written_bits, ndwl * C);
  r.e_write = e_wl + wbits * c_bl * v2 + (ndwl * C - wbits) * c_bl * t.vdd * vsw + e_dec + e_ht;
  // delay proxy: wordline RC + bitline discharge + H-tree wire RC (arbitrary
  // but consistent units, used only to rank organisations)
  const double cell_i = 25.0 * (t.c_gate / 0.85);  // uA read current
  r.t = 1e-3 * C * c_wl_cell * 2.0 + R * c_bl_cell * vsw / cell_i + 1e-6 * L * L * 0.4 +
        0.02 * ilog2(rows_total);
  r.area_um2 = area;
  const double cells = rows_total * cols_total;
  r.leak_w = cells * t.i_leak * kNano * (1.5 * F * 2.0) * t.vdd * 1.3;
  r.rows = (uint32_t)R;
  r.cols = (uint32_t)C;
  return r;
}

}  // namespace

TechParams TechParams::for_node(double nm, double vdd_override) {
  const int n = (int)(sizeof(kNodes) / sizeof(kNodes[0]));
  nm = std::max(kNodes[n - 1].nm, std::min(kNodes[0].nm, nm));
  int i = 0;
  while (i + 1 < n && kNodes[i + 1].nm >= nm) ++i;
  const Node& a = kNodes[i];
  const Node& b = kNodes[std::min(i + 1, n - 1)];
  const double f = (a.nm == b.nm) ? 0.0 : (std::log(a.nm) - std::log(nm)) / (std::log(a.nm) - std::log(b.nm));
  auto lerp = [&](double x, double y) { return x + (y - x) * f; };
  TechParams t;
  t.node_nm = nm;
  t.vdd = vdd_override > 0 ? vdd_override : lerp(a.vdd, b.vdd);
  t.c_gate = lerp(a.c_gate, b.c_gate);
  t.c_wire = lerp(a.c_wire, b.c_wire);
  t.i_leak = lerp(a.i_leak, b.i_leak);
  t.sram_cell_um2 = std::exp(lerp(std::log(a.cell), std::log(b.cell)));
  return t;
}

// CACTI-style search: every (ndwl, ndbl, nspd) whose subarrays stay within
// 32..512 rows and 64..1024 columns; minimum energy x delay of a read
ArrayResult model_array(const ArrayGeom& g, const TechParams& t) {
  ArrayResult out;
  out.name = g.name;
  if (g.bytes <= 0 || g.line_bytes == 0) return out;
  const double bank_bytes = g.bytes / std::max<uint32_t>(1, g.banks);
  const uint32_t assoc = std::max<uint32_t>(1, g.assoc);
  const double sets = std::max(1.0, bank_bytes / ((double)g.line_bytes * assoc));
  const uint32_t ways_read = g.sequential ? 1u : assoc;
  const double line_bits = 8.0 * g.line_bytes;
  double best = -1;
  SubEval bd{};
  for (uint32_t nspd = 1; nspd <= 16; nspd *= 2) {
    const double rows_total = sets * (g.sequential ? assoc : 1) / nspd;
    const double cols_total = line_bits * (g.sequential ? 1 : assoc) * nspd;
    if (rows_total < 1) break;
    for (uint32_t ndwl = 1; ndwl <= 64; ndwl *= 2)
      for (uint32_t ndbl = 1; ndbl <= 64; ndbl *= 2) {
        const double R = rows_total / ndbl, C = cols_total / ndwl;
        if (R < 32 && ndbl > 1) continue;
        if (C < 64 && ndwl > 1) continue;
        if (R > 512 || C > 1024) continue;
        const SubEval e = eval_org(t, rows_total, cols_total, ndwl, ndbl, line_bits * ways_read,
                                   (double)g.out_bits, (double)g.out_bits);
        const double ed = e.e_read * e.t;
        if (best < 0 || ed < best) {
          best = ed;
          bd = e;
          out.ndwl = ndwl;
          out.ndbl = ndbl;
          out.nspd = nspd;
        }
      }
  }
  if (best < 0) {  // tiny array: one subarray
    bd = eval_org(t, std::max(1.0, sets), line_bits * assoc, 1, 1, line_bits * ways_read, (double)g.out_bits,
                  (double)g.out_bits);
    out.ndwl = out.ndbl = out.nspd = 1;
  }
  out.sub_rows = bd.rows;
  out.sub_cols = bd.cols;
  double tag_e = 0, tag_area = 0, tag_leak = 0;
  if (g.tag_bits) {
    // tag array: every way's tag of the set read in parallel, one comparator per way
    const SubEval te = eval_org(t, sets, (double)g.tag_bits * assoc, 1, std::max<uint32_t>(1, (uint32_t)(sets / 256)),
                                (double)g.tag_bits * assoc, (double)g.tag_bits, (double)g.tag_bits);
    tag_e = te.e_read + assoc * g.tag_bits * 2.0 * e_gate(t);
    tag_area = te.area_um2;
    tag_leak = te.leak_w;
  }
  out.e_tag_nj = tag_e / kNano;
  out.e_read_nj = (bd.e_read + tag_e) / kNano;
  out.e_write_nj = (bd.e_write + tag_e) / kNano;
  out.leak_w = (bd.leak_w + tag_leak) * std::max<uint32_t>(1, g.banks);
  out.area_mm2 = (bd.area_um2 + tag_area) * std::max<uint32_t>(1, g.banks) * 1e-6;
  out.t_access_ns = bd.t;
  return out;
}

ArchEnergy arch_energy(const SimCfg& c, const ArchEnergyParams& p) {
  ArchEnergy r;
  const TechParams t = TechParams::for_node(p.node_nm, p.vdd);
  r.tech = t;
  const uint32_t warp = c.warp_size ? c.warp_size : 32;
  const double eg = e_gate(t) / kNano;  // nJ
  auto cache_tag_bits = [](const CacheGeom& g) -> uint32_t {
    const double sets = std::max<uint32_t>(1, g.nsets), line = std::max<uint32_t>(1, g.line);
    const int tb = 48 - ilog2(sets) - ilog2(line);
    return (uint32_t)std::max(8, tb + 2) + (g.sectored ? 4u : 0u);  // + valid/dirty, sector bits
  };
  auto cache_bytes = [](const CacheGeom& g) { return (double)g.nsets * g.assoc * g.line; };
  // ---- per-SM arrays ----
  ArrayGeom l1;
  l1.name = "L1D";
  const double l1_bytes = c.unified_l1_kb ? c.unified_l1_kb * 1024.0 : cache_bytes(c.l1) + c.shmem_per_sm;
  l1.bytes = std::max(cache_bytes(c.l1), 1024.0);
  l1.line_bytes = c.l1.line ? c.l1.line : 128;
  l1.assoc = c.l1.assoc ? c.l1.assoc : 4;
  l1.out_bits = 8 * l1.line_bytes;
  l1.tag_bits = cache_tag_bits(c.l1);
  l1.banks = std::max<uint32_t>(1, c.l1_banks);
  const ArrayResult L1 = model_array(l1, t);
  ArrayGeom sh;
  sh.name = "shared memory";
  sh.bytes = std::max<double>(c.shmem_per_sm, 1024.0);
  sh.line_bytes = 4;
  sh.assoc = 1;
  sh.out_bits = 32;
  sh.banks = std::max<uint32_t>(1, c.smem_banks);
  const ArrayResult SH = model_array(sh, t);
  ArrayGeom il1;
  il1.name = "L1I";
  il1.bytes = std::max(cache_bytes(c.il1), 1024.0);
  il1.line_bytes = c.il1.line ? c.il1.line : 128;
  il1.assoc = c.il1.assoc ? c.il1.assoc : 4;
  il1.out_bits = 128;  // a fetch block
  il1.tag_bits = cache_tag_bits(c.il1);
  const ArrayResult IL1 = model_array(il1, t);
  ArrayGeom cl1;
  cl1.name = "constant cache";
  cl1.bytes = std::max(cache_bytes(c.cl1), 1024.0);
  cl1.line_bytes = c.cl1.line ? c.cl1.line : 64;
  cl1.assoc = c.cl1.assoc ? c.cl1.assoc : 2;
  cl1.out_bits = 32;
  cl1.tag_bits = cache_tag_bits(c.cl1);
  const ArrayResult CL1 = model_array(cl1, t);
  ArrayGeom rf;
  rf.name = "register file";
  rf.bytes = 4.0 * std::max<uint32_t>(c.regs_per_sm, 1024);
  rf.line_bytes = 4 * warp;  // one warp register per row
  rf.assoc = 1;
  rf.out_bits = 32 * warp;
  rf.banks = std::max<uint32_t>(1, c.reg_banks);
  const ArrayResult RF = model_array(rf, t);
  ArrayGeom ib;
  ib.name = "instruction buffer";
  ib.bytes = 16.0 * std::max<uint32_t>(c.max_warps_per_sm, 1) * 2;
  ib.line_bytes = 16;
  ib.assoc = 1;
  ib.out_bits = 64;
  const ArrayResult IB = model_array(ib, t);
  // ---- per-sub-partition L2 slice ----
  ArrayGeom l2;
  l2.name = "L2 slice";
  l2.bytes = std::max(cache_bytes(c.l2), 4096.0);
  l2.line_bytes = c.l2.line ? c.l2.line : 128;
  l2.assoc = c.l2.assoc ? c.l2.assoc : 16;
  l2.out_bits = 256;  // one 32 B sector per access
  l2.tag_bits = cache_tag_bits(c.l2);
  l2.sequential = true;
  const ArrayResult L2 = model_array(l2, t);
  r.arrays = {L1, SH, IL1, CL1, RF, IB, L2};
  (void)l1_bytes;
  // ---- logic ----
  const uint32_t nsched = c.n_sched ? c.n_sched : 1;
  const double warps_per_sched = (double)std::max<uint32_t>(c.max_warps_per_sm, 1) / nsched;
  // scheduler: ready / scoreboard check over its warps + priority arbiter
  const double e_sched = (warps_per_sched * 60.0 + 12.0 * ilog2(warps_per_sched) * 8.0 + 1000.0) * eg;
  const double e_decode = 2000.0 * eg;
  // per lane operation: operand latches and the bypass network around the
  // arithmetic (three 32-bit operands, ~6 gates per latch bit)
  const double e_lane = 3.0 * 32.0 * 6.0 * eg;
  const double e_pipe = 2.0 * 64.0 * 6.0 * eg;  // two 64-bit pipeline registers per stage crossing, ~6 gates per flop
  const double sm_logic_mm2 = 1.0 * (t.node_nm / 12.0) * (t.node_nm / 12.0) * (warp / 32.0) * 6.0;
  r.sm_area_mm2 = L1.area_mm2 + SH.area_mm2 + IL1.area_mm2 + CL1.area_mm2 + RF.area_mm2 + IB.area_mm2 + sm_logic_mm2;
  r.l2_area_mm2 = L2.area_mm2 * c.n_subpart;
  r.die_mm2 = (r.sm_area_mm2 * c.n_sm + r.l2_area_mm2) * 1.25;
  r.leak_sm_w = (L1.leak_w + SH.leak_w + IL1.leak_w + CL1.leak_w + RF.leak_w + IB.leak_w) * c.n_sm;
  r.leak_l2_w = L2.leak_w * c.n_subpart;
  // interconnect: a flit crosses about half the die plus the crossbar switch
  const double flit_bits = 8.0 * (c.flit_size ? c.flit_size : 32);
  const double wire_um = 0.5 * std::sqrt(r.die_mm2) * 1e3;
  const double e_flit = flit_bits * (wire_um * t.c_wire * kFemto * t.vdd * t.vdd * 0.5 / kNano +
                                     2.0 * 6.0 * eg +  // input / output buffer write + read
                                     (double)ilog2(c.n_clusters + c.n_subpart) * 2.0 * eg);
  const double macs = p.tensor_macs_per_lane > 0 ? p.tensor_macs_per_lane : (warp >= 64 ? 128.0 : 32.0);
  double* e = r.base_nj;
  e[PA_TOT_INST] = IB.e_read_nj + e_decode;
  e[PA_FP_INT] = e_sched;
  e[PA_IC_H] = IL1.e_read_nj;
  e[PA_IC_M] = IL1.e_tag_nj + IL1.e_write_nj;  // tag probe + line fill
  e[PA_DC_RH] = L1.e_read_nj;
  e[PA_DC_RM] = L1.e_tag_nj + L1.e_write_nj;  // miss: tag probe, later the fill
  e[PA_DC_WH] = L1.e_write_nj;
  e[PA_DC_WM] = L1.e_tag_nj;  // write-no-allocate: the probe only
  e[PA_CC_H] = CL1.e_read_nj;
  e[PA_CC_M] = CL1.e_tag_nj + CL1.e_write_nj;
  // a warp's shared-memory access: every bank once + the lane crossbar
  e[PA_SHRD_ACC] = SH.e_read_nj * sh.banks + (double)warp * 32.0 * ilog2(sh.banks) * eg;
  e[PA_REG_RD] = RF.e_read_nj;
  e[PA_REG_WR] = RF.e_write_nj;
  e[PA_INT_ACC] = op_nj(kIntAdd, t) + e_lane;
  e[PA_INT_MUL_ACC] = op_nj(kIntMul, t) + e_lane;
  e[PA_FP_ACC] = op_nj(kFpAdd + kFpMul, t) + e_lane;  // an fp32 FMA
  e[PA_FP_MUL_ACC] = op_nj(kFpMul, t) + e_lane;
  e[PA_DP_ACC] = op_nj(kDpAdd + kDpMul, t) + 2.0 * e_lane;
  e[PA_DP_MUL_ACC] = op_nj(kDpMul, t) + 2.0 * e_lane;
  e[PA_FP_SQRT_ACC] = e[PA_FP_LG_ACC] = e[PA_FP_SIN_ACC] = e[PA_FP_EXP_ACC] = op_nj(kSfu, t) + e_lane;
  e[PA_TENSOR_ACC] = macs * op_nj(kMac16, t) + e_lane;
  e[PA_TEX_ACC] = L1.e_read_nj;  // a texture fetch reads the (unified) L1 array
  e[PA_MEM_RD] = p.dram_pj_per_bit * 256.0 * 1e-3;  // one 32 B column access
  e[PA_MEM_WR] = p.dram_pj_per_bit * 256.0 * 1e-3 * 1.1;
  e[PA_MEM_PRE] = p.dram_act_nj;
  e[PA_L2_RH] = L2.e_read_nj;
  e[PA_L2_RM] = L2.e_tag_nj + L2.e_write_nj;  // probe + the sector fill
  e[PA_L2_WH] = L2.e_write_nj;
  e[PA_L2_WM] = L2.e_tag_nj + L2.e_write_nj;  // write-allocate of the written sectors
  e[PA_NOC_A] = e_flit;
  e[PA_PIPE_A] = e_pipe;
  return r;
}

std::string arch_energy_report(const ArchEnergy& e) {
  std::ostringstream o;
  char b[256];
  snprintf(b, sizeof(b), "technology: %.1f nm, Vdd %.3f V, SRAM cell %.4f um^2\n", e.tech.node_nm, e.tech.vdd,
           e.tech.sram_cell_um2);
  o << b;
  o << "array                  read_nJ   write_nJ    tag_nJ   leak_mW   area_mm2  ndwl ndbl nspd  rows cols\n";
  for (const auto& a : e.arrays) {
    snprintf(b, sizeof(b), "%-20s %9.5f %10.5f %9.5f %9.3f %10.4f %5u %4u %4u %5u %4u\n", a.name.c_str(),
             a.e_read_nj, a.e_write_nj, a.e_tag_nj, a.leak_w * 1e3, a.area_mm2, a.ndwl, a.ndbl, a.nspd, a.sub_rows,
             a.sub_cols);
    o << b;
  }
  snprintf(b, sizeof(b), "SM %.3f mm^2, L2 %.2f mm^2, die estimate %.1f mm^2; array leakage SMs %.1f W, L2 %.1f W\n",
           e.sm_area_mm2, e.l2_area_mm2, e.die_mm2, e.leak_sm_w, e.leak_l2_w);
  o << b;
  return o.str();
}

}  // namespace asim
