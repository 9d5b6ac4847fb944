// Device side of the MI355X (gfx950) cycle engine: the persistent
// engine_kernel and its helpers.  Included by the kernel translation units
// (engine_k_*.hip: each instantiates a few builds of the kernel, so they
// compile in parallel) and, for the shared declarations, by gpu_engine.hip
// (the host side).
//
// One persistent launch simulates up to `max_epochs` PDES epochs of the whole
// simulated GPU:
//   * block b < n_sm      : one 64-lane wavefront owns SM b (LDS-state build:
//                           its complete SMState lives in LDS for the launch;
//                           global-state build: simulated in place in HBM).
//   * block n_sm + c      : one wavefront owns memory channel c (two L2
//                           sub-partitions + the DRAM channel).
//   * after every epoch   : one grid-wide barrier (agent-scope release /
//                           acquire, XCD-local counters first, then a global
//                           generation word), then every block evaluates the
//                           same epoch decision and all blocks leave together.
// The cycle model itself is the shared single-source code in csrc/model, run
// with the WavePar lane policy, so results are bit-identical to the CPU
// reference engine.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"
#include "grid_barrier.h"
#include "wave_par.h"
#include "sm_split.h"

namespace asim {

// The configuration of every running simulation lives in constant memory
// (one slot per engine instance of the process, GpuArgs::cfg_slot).  Read
// through address space 4, every wave-uniform access is a scalar load the
// compiler may hoist and CSE freely (constant memory is never written by a
// kernel), so configuration-derived values stay in SGPRs and their
// arithmetic is SALU; only lane-indexed reads become vector loads.  From the
// LDS copy used before, each read after any state store had to be re-issued
// (the compiler cannot rule out aliasing with the state in LDS) and landed in
// a VGPR: constant memory measured 6-7 % faster on bfs / hotspot / heartwall
// (profiles/r4/ab_cfg_const_vs_lds.txt), bit-exact.
constexpr int kCfgSlots = 64;
// (internal linkage: every kernel translation unit has its own copy, which
// its engine_upload_cfg_* function fills -- engine_k_common.h)
static __constant__ SimCfg g_cfg[kCfgSlots];

// in-kernel power sampler state (engine.h PwrArm; power_eval.h)
struct PwrDev {
  PwrCoef coef;
  uint64_t freq;
  uint64_t t_prev;  // cycle of the previous sample (evaluator block)
  uint64_t next;    // next sample point (written back by block 0 at exit)
  uint32_t n_sm;
  uint32_t n;       // samples written to `ring` this launch
  uint32_t cap;
  uint32_t pad;
  double s_prev[kPwrSumPad];
  double* rows;      // [units][kPwrRawPad] raw counters of the sample being taken
  PwrSample* ring;   // [cap] samples of this launch (the host drains after it)
};

struct GpuArgs {
  uint32_t cfg_slot;                 // g_cfg slot of this engine
  const SimCfg* __restrict__ cfg_g;  // global copy (not read by the engine kernel)
  const KernelTab* kt;               // running kernels (copied into LDS at launch)
  SMState* sms;
  ChanState* chs;
  EpochPub* pub;
  Pkt* box_req[2];
  uint32_t* cnt_req[2];
  Pkt* box_rep[2];
  uint32_t* cnt_rep[2];
  uint32_t cap_req, cap_rep;
  Pkt* ovf;
  uint32_t ovf_cap;
  L2Line* mall;  // [n_mem][mall_sets * mall_assoc] or nullptr
  uint64_t* link_free;  // -icnt_link_contention: [links] free times, then 2 statistics words; or nullptr
  uint32_t* link_refs;  // the pass's packet list
  uint64_t epoch0;
  uint64_t cycle0;
  uint64_t max_cycle;
  uint32_t max_epochs;
  uint32_t nblocks;
  uint32_t block0;  // batch launch: the simulation's first block in the grid (0 otherwise)
  uint32_t ch_blocks;  // split build: blocks of the channels (the last ones; 0: units round-robin over all blocks)
  GpuCtl* ctl;
  uint64_t* prof;  // [nblocks][kProfSlots] shader-clock cycles per stage (profiling build)
  uint32_t* ework; // [nblocks] work clocks of the last epoch (profiling build)
  PwrDev* pw;      // armed power sampler, or nullptr
};

template <class T>
__device__ __forceinline__ void copy_state(T* dst, const T* src) {
  static_assert(sizeof(T) % 16 == 0, "state must be 16-byte granular");
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const int n = (int)(sizeof(T) / 16);
  for (int i = (int)(threadIdx.x & 63); i < n; i += 64) d[i] = s[i];
  __syncthreads();
}

// HBM -> LDS state swap-in for time-sliced units: LDS-DMA (global_load_lds,
// 16 B per lane, lane-linear LDS image) issues the whole state back to back
// with no VGPR staging, then one wait.
template <class T>
__device__ __forceinline__ void swap_in(T* lds, const T* src) {
  static_assert(sizeof(T) % 16 == 0, "state must be 16-byte granular");
  typedef __attribute__((address_space(1))) const uint4 g4;
  typedef __attribute__((address_space(3))) uint4 l4;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(lds);
  const int n = (int)(sizeof(T) / 16);
  const int lane = (int)(threadIdx.x & 63);
  for (int i = 0; i < n; i += 64)
    if (i + lane < n) __builtin_amdgcn_global_load_lds((g4*)(s + i + lane), (l4*)(d + i), 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}
// LDS -> HBM swap-out: eight 16-byte LDS reads in flight per lane, then the
// stores (completion is awaited by the epoch barrier's release fence)
template <class T>
__device__ __forceinline__ void swap_out(T* dst, const T* lds) {
  const uint4* s = reinterpret_cast<const uint4*>(lds);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const int n = (int)(sizeof(T) / 16);
  const int lane = (int)(threadIdx.x & 63);
  int i = 0;
  for (; i + 4 * 64 <= n; i += 4 * 64) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = s[i + j * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) d[i + j * 64 + lane] = v[j];
  }
  for (; i < n; i += 64)
    if (i + lane < n) d[i + lane] = s[i + lane];
  __syncthreads();
}

// the first `bytes` (a multiple of 16) of a state, HBM <-> LDS (split-state
// build: the SM's hot prefix)
__device__ __forceinline__ void copy_bytes(void* dst, const void* src, size_t bytes) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const int n = (int)(bytes / 16);
  for (int i = (int)(threadIdx.x & 63); i < n; i += 64) d[i] = s[i];
  __syncthreads();
}

extern __shared__ __attribute__((aligned(16))) char g_lds[];
// Block LDS layout: the kernel table, the stage profiler and the power
// evaluator's scratch first (a few KB), then -- in the LDS-state build -- the
// resident unit's state.  The global-state build (ASIM_GPU_STATE=global)
// allocates only the first part: its units work on their HBM images, so many
// engine waves share a CU.
constexpr int kProfSlots = 56;
struct ProfLds {
  uint64_t last;
  uint32_t slot;
  uint32_t pad;
  uint64_t acc[kProfSlots];
};
constexpr size_t kKtOff = 0;
constexpr size_t kProfOff = kKtOff + (sizeof(KernelTab) + 15) / 16 * 16;
// the power evaluator's sums and deltas (one block per sample)
constexpr size_t kPwrOff = kProfOff + (sizeof(ProfLds) + 15) / 16 * 16;
constexpr size_t kStateOff = (kPwrOff + 2 * kPwrSumPad * sizeof(double) + 15) / 16 * 16;
constexpr size_t kStateLds = ((sizeof(SMState) > sizeof(ChanState) ? sizeof(SMState) : sizeof(ChanState)) + 15) / 16 * 16;
constexpr size_t kLdsBytes = kStateOff + kStateLds;
constexpr size_t kLdsBytesGlobal = kStateOff;
constexpr size_t kLdsBytesSplit = kStateOff + kSmHotBytes;
// engine builds: the unit state's home during a launch
enum EngineMode : int {
  kModeLds = 0,     // whole unit state in LDS (one block per CU)
  kModeGlobal = 1,  // every unit in place in HBM
  kModeSplit = 2,   // SM: hot prefix in LDS, geometry-sized arrays in HBM (SmSplit); channels in place in HBM
};
static_assert(kLdsBytes <= 160 * 1024, "per-block LDS budget exceeded");

// a pointer the compiler may treat as global memory (address space 1): the
// generic -> global cast lets address-space inference turn the model's flat
// accesses through it into global_load / global_store
template <class T>
__device__ __forceinline__ T* as_global(T* p) {
  typedef __attribute__((address_space(1))) T gT;
  return (T*)(gT*)p;
}

// profiling build of the lane policy: P::prof(k) charges the shader-clock
// time since the previous stamp to the previous stage and enters stage k
struct WaveParProf : WavePar {
  static __device__ __forceinline__ void prof(int k) {
    ProfLds* p = reinterpret_cast<ProfLds*>(g_lds + kProfOff);
    uint64_t t = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
      p->acc[p->slot] += t - p->last;
      p->slot = (uint32_t)k;
      p->last = t;
    }
    __builtin_amdgcn_wave_barrier();
  }
  // event counters in the spare slots (not time): P::tick(k) adds one
  static __device__ __forceinline__ void tick(int k) {
    ProfLds* p = reinterpret_cast<ProfLds*>(g_lds + kProfOff);
    if ((threadIdx.x & 63) == 0) p->acc[k] += 1;
    __builtin_amdgcn_wave_barrier();
  }
};

typedef double f64x4 __attribute__((ext_vector_type(4)));

// a unit's raw power counters (power_eval.h step 1) into its row
__device__ __forceinline__ void pwr_row_sm(double* row, const SMStats& st) {
  for (int k = (int)(threadIdx.x & 63); k < kPwrRawPad; k += 64) row[k] = k < PR_COUNT ? (double)pwr_raw_sm(st, k) : 0.0;
}
__device__ __forceinline__ void pwr_row_ch(double* row, const ChanState& ch, uint32_t nsub) {
  for (int k = (int)(threadIdx.x & 63); k < kPwrRawPad; k += 64) {
    double v = 0;
    if (k < PR_COUNT)
      for (uint32_t j = 0; j < nsub; ++j) v += (double)pwr_raw_mem(ch.sp[j].st, k);
    row[k] = v;
  }
}

// power_eval.h steps 2 and 3 on one wave: S = rows x M as f64 MFMA tiles
// (16 units x 4 raw counters by 4 raw counters x 16 sums, accumulated over
// unit tiles and k-steps; integers below 2^53, so exact in any order), then
// the sample on lane 0 into the ring
__device__ void pwr_evaluate(PwrDev& pw, uint32_t nunits, uint64_t now) {
  const int lane = (int)(threadIdx.x & 63);
  constexpr int kCt = kPwrSumPad / 16;
  f64x4 acc[kCt];
#pragma unroll
  for (int ct = 0; ct < kCt; ++ct) acc[ct] = f64x4{0.0, 0.0, 0.0, 0.0};
  const double* rows = pw.rows;
  for (uint32_t t = 0; t < (nunits + 15u) / 16u; ++t) {
    const uint32_t u = 16u * t + (uint32_t)(lane & 15);
    for (int k4 = 0; k4 < kPwrRawPad / 4; ++k4) {
      const int k = 4 * k4 + (lane >> 4);
      const double av = u < nunits ? rows[(size_t)u * kPwrRawPad + k] : 0.0;
      const int sj = k < PR_COUNT ? pwr_sum_of(k) : -1;
#pragma unroll
      for (int ct = 0; ct < kCt; ++ct) {
        const double bv = sj == 16 * ct + (lane & 15) ? 1.0 : 0.0;
        acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[ct], 0, 0, 0);
      }
    }
  }
  double* S = reinterpret_cast<double*>(g_lds + kPwrOff);
  double* D = S + kPwrSumPad;
#pragma unroll
  for (int ct = 0; ct < kCt; ++ct) {
    // D layout: column lane & 15, rows (lane >> 4) + 4 * reg: sum the four
    // rows a lane holds, then across the four lane groups
    double v = acc[ct][0] + acc[ct][1] + acc[ct][2] + acc[ct][3];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 16) S[16 * ct + lane] = v;
  }
  __syncthreads();
  if (lane < PS_COUNT) D[lane] = S[lane] - pw.s_prev[lane];
  __syncthreads();
  if (lane == 0) {
    const uint32_t i = pw.n < pw.cap ? pw.n : pw.cap - 1;
    PwrSample& o = pw.ring[i];
    pwr_activity(D, now > pw.t_prev ? (double)(now - pw.t_prev) : 1.0, pw.n_sm, o);
    pwr_power(pw.coef, pw.coef.coef, pw.n_sm, 1.0, 1.0, 1.0, o);
    o.now = now;
    pw.t_prev = now;
    pw.n = pw.n + 1;
  }
  if (lane < PS_COUNT) pw.s_prev[lane] = S[lane];
  __syncthreads();
}

// the kernel body for block `b` of the simulation `a` (b = blockIdx.x for a
// single simulation; a batch launch maps its blocks onto several)
template <class P, bool kSliced, int kMode>
__device__ __forceinline__ void engine_body(const GpuArgs& a, const uint32_t b) {
  constexpr bool kGlobal = kMode == kModeGlobal, kSplit = kMode == kModeSplit;
  // The configuration is read all over the model, much of it at lane-varying
  // indices (address-decoder bit runs, per-unit counts, cache geometries
  // selected per warp): constant memory, one slot per engine (g_cfg above).
  const SimCfg& c = g_cfg[a.cfg_slot];
  const uint64_t E = c.icnt_latency;
  // Units (SMs 0..n_sm-1, then channels) map to blocks round-robin: unit
  // b + k * nblocks.  LDS-state build: with no more units than blocks each
  // block owns one unit whose state stays in LDS for the whole launch;
  // otherwise (configs larger than the CU count, e.g. the 384-unit MI355X
  // preset) a block time-slices its units every epoch, swapping states
  // through HBM and keeping the last one resident into the next epoch.
  // Global-state build (kGlobal): every unit is simulated in place in its HBM
  // image (vector-L1 / L2 resident while its block works on it), the block
  // holds no state in LDS and several engine waves share each CU.
  // Split-state build (kSplit): an SM's hot prefix is in LDS (swapped like a
  // whole state when time-sliced), its tail and every channel in HBM.
  SMState* s = reinterpret_cast<SMState*>(g_lds + kStateOff);
  ChanState* ch = reinterpret_cast<ChanState*>(g_lds + kStateOff);
  const uint32_t nunits = c.n_sm + c.n_mem;
  // With a.ch_blocks, the SMs spread over the first blocks and the channels
  // over the last a.ch_blocks (several channels per block: a channel's epoch
  // is a fraction of an SM's, so packing them leaves the critical path alone
  // and frees CUs for other simulations); otherwise unit b + k * nblocks.
  const uint32_t nsmb = a.nblocks - a.ch_blocks;
  auto unit_k = [&](uint32_t k) -> uint32_t {
    if (!a.ch_blocks) return b + k * a.nblocks;
    return b < nsmb ? b + k * nsmb : c.n_sm + (b - nsmb) + k * a.ch_blocks;
  };
  const uint32_t nmine = !kSliced ? 1u
                         : !a.ch_blocks ? (nunits - 1 - b) / a.nblocks + 1
                         : b < nsmb ? (c.n_sm - 1 - b) / nsmb + 1
                                    : (c.n_mem - 1 - (b - nsmb)) / a.ch_blocks + 1;
  const uint32_t u0 = unit_k(0);
  uint32_t loaded = u0;  // unit whose state is in LDS (global build: the unit being simulated)
  auto bind = [&](uint32_t u) {
    if (u < c.n_sm) s = as_global(&a.sms[u]);
    else ch = as_global(&a.chs[u - c.n_sm]);
  };
  uint32_t hot = u0;  // split build: the SM whose hot prefix is in LDS (~0u: none)
  auto swap_to = [&](uint32_t u) {
    if (kGlobal) {
      bind(u);
      loaded = u;
      return;
    }
    if (kSplit) {
      loaded = u;
      if (u >= c.n_sm) {
        ch = as_global(&a.chs[u - c.n_sm]);
        return;
      }
      if (u == hot) return;
      if (hot < c.n_sm) copy_bytes(&a.sms[hot], s, kSmHotBytes);
      copy_bytes(s, &a.sms[u], kSmHotBytes);
      hot = u;
      return;
    }
    if (!kSliced || u == loaded) return;
    if (loaded < c.n_sm) swap_out(&a.sms[loaded], s);
    else swap_out(&a.chs[loaded - c.n_sm], ch);
    if (u < c.n_sm) swap_in(s, &a.sms[u]);
    else swap_in(ch, &a.chs[u - c.n_sm]);
    loaded = u;
  };
  if (kGlobal)
    bind(u0);
  else if (kSplit && u0 < c.n_sm)
    copy_bytes(s, &a.sms[u0], kSmHotBytes);
  else if (kSplit) {
    hot = ~0u;
    ch = as_global(&a.chs[u0 - c.n_sm]);
  } else if (u0 < c.n_sm)
    copy_state(s, &a.sms[u0]);
  else
    copy_state(ch, &a.chs[u0 - c.n_sm]);
  // kernel table lives in LDS (never in scratch)
  KernelTab* ktl = reinterpret_cast<KernelTab*>(g_lds + kKtOff);
  {
    static_assert(sizeof(KernelTab) % 16 == 0, "kernel table must be 16-byte granular");
    const uint4* src = reinterpret_cast<const uint4*>(a.kt);
    uint4* dst = reinterpret_cast<uint4*>(ktl);
    for (int i = (int)(threadIdx.x & 63); i < (int)(sizeof(KernelTab) / 16); i += 64) dst[i] = src[i];
  }
  ProfLds* pl = reinterpret_cast<ProfLds*>(g_lds + kProfOff);
  if ((threadIdx.x & 63) == 0) {
    pl->last = __builtin_amdgcn_s_memtime();
    pl->slot = 31;
    for (int i = 0; i < kProfSlots; ++i) pl->acc[i] = 0;
  }
  __syncthreads();
  const KernelTab& kt = *ktl;
  SmCtx sx;
  sx.cfg = &c;
  sx.kt = &kt;
  sx.out_cap = a.cap_req;
  sx.n_src_sm = c.n_sm;
  sx.rt_st = c.link_contention == 2 ? a.link_free : nullptr;
  MemCtx mx;
  mx.cfg = &c;
  mx.out_cap = a.cap_rep;
  mx.n_src_sub = c.n_subpart;
  mx.ovf = a.ovf;
  mx.ovf_cap = a.ovf_cap;
  mx.rt_st = c.link_contention == 2 ? a.link_free : nullptr;
  mx.mall = nullptr;
  uint64_t epoch = a.epoch0, cycle = a.cycle0;
  uint64_t t_work0 = a.ework ? __builtin_amdgcn_s_memtime() : 0;
  uint32_t done = 0, dead = 0, capped = 0;
  uint32_t n = 0;
  uint32_t nbar = 0;  // grid barriers of this launch (epochs + power samples)
  uint64_t pw_next = a.pw ? a.pw->next : 0;
  bool failed = false;
  // destinations with packets in the previous epoch's mailboxes (all at the
  // launch's first epoch): the gathers of the others are skipped
  uint64_t reqm[2] = {~0ull, ~0ull}, repm[2] = {~0ull, ~0ull};
  for (; n < a.max_epochs;) {
    const uint32_t cur = (uint32_t)(epoch & 1), prev = cur ^ 1u;
    const uint64_t t0 = cycle, t1 = t0 + E;
    // the resident unit first, then the others (units are independent
    // within an epoch: they read only the previous epoch's mailboxes)
    uint32_t first_k = 0;
    for (uint32_t k = 0; k < nmine; ++k)
      if (unit_k(k) == loaded) first_k = k;
    for (uint32_t j = 0; j < nmine; ++j) {
      const uint32_t u = unit_k((first_k + j) % nmine);
      swap_to(u);
      if (u < c.n_sm) {
        sx.outbox = a.box_req[cur];
        sx.outcnt = a.cnt_req[cur];
        if constexpr (kSplit) {
          SmSplit sp(*s, *as_global(&a.sms[u]));
          sm_epoch<P>(sp, sx, *a.pub, prev, t0, t1, a.box_rep[prev], a.cnt_rep[prev], a.cap_rep, c.n_subpart, epoch,
                      repm);
          sm_publish<P>(sp, sx, *a.pub, cur);
        } else {
          sm_epoch<P>(*s, sx, *a.pub, prev, t0, t1, a.box_rep[prev], a.cnt_rep[prev], a.cap_rep,
                      c.n_subpart, epoch, repm);
          sm_publish<P>(*s, sx, *a.pub, cur);
        }
      } else {
        mx.outbox = a.box_rep[cur];
        mx.outcnt = a.cnt_rep[cur];
        mx.mall = a.mall ? a.mall + (size_t)(u - c.n_sm) * ((size_t)c.mall_sets * c.mall_assoc) : nullptr;
        mx.win_end = core_fs(c, t1);
        chan_epoch<P>(*ch, mx, a.box_req[prev], a.cnt_req[prev], a.cap_req, core_fs(c, t0), reqm);
        chan_publish<P>(*ch, mx, *a.pub, cur);
      }
    }
    ++n;
    P::prof(26);  // barrier
    uint64_t t_arrive = 0;
    if (a.ework) {
      t_arrive = __builtin_amdgcn_s_memtime();
      if ((threadIdx.x & 63) == 0) a.ework[b] = (uint32_t)(t_arrive - t_work0);
    }
    uint32_t was_last = 0;
    if (!grid_barrier_b(a.ctl, b, a.nblocks, nbar++, &was_last)) break;
    if (a.link_free) {
      // shared links of multi-hop routes: block 0 walks this epoch's packets
      // in the fixed order (icnt_links.h), then every block waits for it
      // before a destination reads them
      if (b == 0)
        icnt_epoch_pass<P>(c, a.box_req[cur], a.cnt_req[cur], a.cap_req, a.box_rep[cur], a.cnt_rep[cur], a.cap_rep,
                           a.link_free, a.link_refs);
      if (!grid_barrier_b(a.ctl, b, a.nblocks, nbar++)) break;
    }
    P::prof(27);  // decision
    if (a.ework) {
      const uint64_t t_exit = __builtin_amdgcn_s_memtime();
      if ((threadIdx.x & 63) == 0 && was_last) { pl->acc[34] += t_exit - t_arrive; pl->acc[35] += 1; }
      if (b == 0) {
        // slowest block's work this epoch (critical path) and the epoch count
        uint64_t mk = 0;  // work << 32 | block: the slowest block and its work
        for (uint32_t j = threadIdx.x & 63; j < a.nblocks; j += 64) {
          const uint64_t k = (uint64_t)a.ework[j] << 32 | j;
          mk = k > mk ? k : mk;
        }
        mk = WavePar::red_max64(mk);
        const uint32_t m = (uint32_t)(mk >> 32);
        if ((threadIdx.x & 63) == 0) {
          pl->acc[32] += m;
          pl->acc[33] += 1;
          // per block: epochs in which it was the slowest (slot 30)
          atomicAdd((unsigned long long*)&a.prof[(size_t)(uint32_t)mk * kProfSlots + 30], 1ull);
        }
      }
      t_work0 = t_exit;
    }
    // an armed power sampler's next point clamps the fast-forward like a
    // sampled slice's max_cycle would
    const uint64_t mc = a.pw ? (a.max_cycle ? (a.max_cycle < pw_next ? a.max_cycle : pw_next) : pw_next) : a.max_cycle;
    EpochDecision d = epoch_decide<P>(c, *a.pub, cur, t1, kt, epoch, mc);
    reqm[0] = P::uni(d.req_dst[0]);
    reqm[1] = P::uni(d.req_dst[1]);
    repm[0] = P::uni(d.rep_dst[0]);
    repm[1] = P::uni(d.rep_dst[1]);
    P::prof(28);
    ++epoch;
    cycle = P::uni(d.next_start);
    if (a.pw) {
      const bool exits = P::uni(d.done) || P::uni(d.deadlock) || P::uni(d.limit) || (a.max_cycle && cycle >= a.max_cycle);
      if (exits || cycle >= pw_next) {
        // every block writes its units' counters, one barrier, then the last
        // block evaluates the sample while the others run on
        for (uint32_t k = 0; k < nmine; ++k) {
          const uint32_t u = unit_k(k);
          double* row = a.pw->rows + (size_t)u * kPwrRawPad;
          if (u < c.n_sm) pwr_row_sm(row, (!kGlobal && u == (kSplit ? hot : loaded)) ? s->st : a.sms[u].st);
          else pwr_row_ch(row, (!kGlobal && !kSplit && u == loaded) ? *ch : a.chs[u - c.n_sm], c.n_sub_per_mem);
        }
        if (!grid_barrier_b(a.ctl, b, a.nblocks, nbar++)) { failed = true; break; }
        if (b == a.nblocks - 1) pwr_evaluate(*a.pw, nunits, cycle);
        pw_next = cycle + a.pw->freq;
      }
    }
    if (P::uni(d.done)) { done = P::uni(d.done); break; }
    if (P::uni(d.deadlock)) { dead = 1; break; }
    if (P::uni(d.limit)) { capped = 1; break; }
    if (P::uni(d.refill)) break;  // the host streams in more of a kernel's trace
    if (a.max_cycle && cycle >= a.max_cycle) break;
  }
  P::prof(31);  // launch_rest
  // write the resident state back
  if (kGlobal)
    ;
  else if (kSplit) {
    if (hot < c.n_sm) copy_bytes(&a.sms[hot], s, kSmHotBytes);
  } else if (loaded < c.n_sm)
    copy_state(&a.sms[loaded], s);
  else
    copy_state(&a.chs[loaded - c.n_sm], ch);
  if (a.prof && (threadIdx.x & 63) < kProfSlots && (threadIdx.x & 63) != 30) a.prof[(size_t)b * kProfSlots + (threadIdx.x & 63)] += pl->acc[threadIdx.x & 63];
  (void)failed;
  if (a.pw && b == 0 && (threadIdx.x & 63) == 0) a.pw->next = pw_next;
  if (b == 0 && (threadIdx.x & 63) == 0) {
    a.ctl->done = done;
    a.ctl->deadlock = dead;
    a.ctl->cap = capped;
    a.ctl->end_cycle = cycle;
    a.ctl->end_epoch = epoch;
    a.ctl->epochs_run = n;
  }
}


// One wave per block and at most one engine wave per SIMD (the LDS-state
// build holds a whole CU's LDS; the global-state build's 256 VGPRs allow one
// wave per SIMD): amdgpu_waves_per_eu(1, 1) lets the register allocator use
// the accumulation registers too, so the engine spills to AGPRs instead of
// scratch memory.
#define ASIM_ENGINE_KERNEL_ATTRS __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))

template <class P, bool kSliced, int kMode>
__global__ void ASIM_ENGINE_KERNEL_ATTRS engine_kernel(GpuArgs a) {
  engine_body<P, kSliced, kMode>(a, blockIdx.x);
}

// Many simulations in one launch (global-state build): block i runs block
// i - jobs[j].block0 of simulation j = block_job[i]; every simulation has its
// own configuration slot, state, mailboxes and grid-barrier counters, so its
// blocks synchronise among themselves only.  One launch hosts as many
// simulations as fit the GPU, past the per-process limit on concurrent
// kernels (GPU_MAX_HW_QUEUES).
__global__ void ASIM_ENGINE_KERNEL_ATTRS engine_batch_kernel(const GpuArgs* __restrict__ jobs,
                                                             const uint16_t* __restrict__ block_job);
// the same for the split-state build
__global__ void ASIM_ENGINE_KERNEL_ATTRS engine_batch_split_kernel(const GpuArgs* __restrict__ jobs,
                                                                   const uint16_t* __restrict__ block_job);

// the split build at two engine waves per SIMD (engine_k_split2.hip)
__global__ void engine_split2_kernel(GpuArgs a);

// the kernel TUs' configuration uploads (one per TU: its own g_cfg)
#define ASIM_ENGINE_CFG_UPLOAD(name)                                                         \
  hipError_t engine_upload_cfg_##name(const SimCfg& c, int slot) {                          \
    return hipMemcpyToSymbol(HIP_SYMBOL(g_cfg), &c, sizeof(SimCfg), sizeof(SimCfg) * (size_t)slot, \
                             hipMemcpyHostToDevice);                                         \
  }

}  // namespace asim
