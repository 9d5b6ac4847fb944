// Register-resident view of one SM's hot state for the cycle loop of an epoch
// on the MI355X engine.
//
// The cycle model (csrc/model/sm.h) is written against SMState, which lives
// in LDS on the GPU.  Measured on MI355X (ub_lds_uniform): a dependent LDS
// access costs ~170 shader clocks, and one simulated SM cycle is a chain of
// ~60-180 of them (the stage early-exit checks, the per-warp readiness
// ballots, the statistics read-modify-writes).  SmView re-exposes every
// SMState member under the same name, so the model code runs unchanged
// (templated on the state type), but
//   * per-warp fields the ballots read every cycle live in one VGPR each
//     (lane w holds warp w: WarpReg<T>),
//   * the scalar bookkeeping fields live in registers (the statistics stay in
//     LDS: promoting them too measured ~1 % slower, SGPR spills),
//   * everything else (instruction windows, caches, rings, queues) stays a
//     reference into the LDS state.
// The view is loaded when an SM's cycle loop starts and flushed back before
// the epoch ends, so SMState stays the single source of truth between epochs
// (snapshots, checkpoints, host reads and the CPU engine are unaffected).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace asim {

__device__ __forceinline__ int sv_lane() { return (int)(threadIdx.x & 63); }

template <class T>
__device__ __forceinline__ T sv_uni(T v) {
  uint64_t u = 0;
  __builtin_memcpy(&u, &v, sizeof(T));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  uint32_t hi = 0;
  if constexpr (sizeof(T) == 8) hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  u = ((uint64_t)hi << 32) | lo;
  T r;
  __builtin_memcpy(&r, &u, sizeof(T));
  return r;
}

// One per-warp field in a VGPR.  Indexing works in both contexts the model
// uses: lane-parallel sections (index == this lane's warp: the lane's own
// register) and wave-uniform code (index in an SGPR: v_readlane / a masked
// write by the owning lane).  Which one applies is decided at run time from
// the index itself (one readfirstlane + ballot).
template <class T>
struct WarpReg {
  T v;
  __device__ __forceinline__ T get(int w) const {
    const int w0 = __builtin_amdgcn_readfirstlane(w);
    if (__builtin_amdgcn_ballot_w64(w != w0) == 0) {
      if constexpr (sizeof(T) == 8) {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, w0);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), w0);
        return (T)(((uint64_t)hi << 32) | lo);
      } else {
        return (T)__builtin_amdgcn_readlane((int)(uint32_t)v, w0);
      }
    }
    return v;
  }
  __device__ __forceinline__ void put(int w, T x) {
    if (sv_lane() == w) v = x;
  }
  struct Ref {
    WarpReg* r;
    int w;
    __device__ __forceinline__ operator T() const { return r->get(w); }
    __device__ __forceinline__ Ref& operator=(T x) {
      r->put(w, x);
      return *this;
    }
    __device__ __forceinline__ Ref& operator=(const Ref& o) {
      r->put(w, (T)o);
      return *this;
    }
    __device__ __forceinline__ Ref& operator+=(T x) { return *this = (T)(r->get(w) + x); }
    __device__ __forceinline__ Ref& operator-=(T x) { return *this = (T)(r->get(w) - x); }
    __device__ __forceinline__ Ref& operator|=(T x) { return *this = (T)(r->get(w) | x); }
    __device__ __forceinline__ Ref& operator&=(T x) { return *this = (T)(r->get(w) & x); }
    __device__ __forceinline__ Ref& operator++() { return *this = (T)(r->get(w) + 1); }
    __device__ __forceinline__ Ref& operator--() { return *this = (T)(r->get(w) - 1); }
    __device__ __forceinline__ T operator++(int) {
      const T o = r->get(w);
      r->put(w, (T)(o + 1));
      return o;
    }
    __device__ __forceinline__ T operator--(int) {
      const T o = r->get(w);
      r->put(w, (T)(o - 1));
      return o;
    }
  };
  __device__ __forceinline__ Ref operator[](int w) { return Ref{this, w}; }
  __device__ __forceinline__ T operator[](int w) const { return get(w); }
  // arrays shorter than the wave: lanes past the end hold 0 and store nothing
  template <class A>
  __device__ __forceinline__ void load(const A& arr) {
    constexpr int n = (int)std::extent<A>::value;
    if constexpr (n >= 64) {
      v = arr[sv_lane()];
    } else {
      v = sv_lane() < n ? arr[sv_lane() < n ? sv_lane() : 0] : (T)0;
    }
  }
  template <class A>
  __device__ __forceinline__ void store(A& arr) const {
    constexpr int n = (int)std::extent<A>::value;
    if (n >= 64 || sv_lane() < n) arr[sv_lane() < n ? sv_lane() : 0] = v;
  }
};

// the scoreboard of this lane's warp: four 64-bit register words per lane
// (csrc/model/sm.h sbt/sbs/sbc/sbz are overloaded for it below)
struct WarpSb {
  uint64_t v[4];
  __device__ __forceinline__ uint64_t word(uint32_t k) const {
    return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
  }
  template <class A>
  __device__ __forceinline__ void load(const A& arr) {
    const int l = sv_lane();
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = arr[l][k];
  }
  template <class A>
  __device__ __forceinline__ void store(A& arr) const {
    const int l = sv_lane();
#pragma unroll
    for (int k = 0; k < 4; ++k) arr[l][k] = v[k];
  }
};
__device__ __forceinline__ bool sbt(const WarpSb& sb, uint32_t w, uint8_t r) {
  if (!r) return false;
  const uint32_t k = (uint32_t)r >> 6;
  uint64_t m = sb.word(k);
  const int w0 = __builtin_amdgcn_readfirstlane((int)w);
  if (__builtin_amdgcn_ballot_w64((int)w != w0) == 0) {  // wave-uniform (warp, register)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, w0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), w0);
    m = ((uint64_t)hi << 32) | lo;
  }
  return (m >> (r & 63)) & 1ull;
}
__device__ __forceinline__ void sb_upd(WarpSb& sb, uint32_t w, uint8_t r, bool set) {
  if (!r) return;
  // the register's word is wave-uniform whenever the register is (the usual
  // case: one warp's instruction): a scalar branch picks the word and one
  // masked VALU op per half updates it; lane-varying registers take the
  // generic select over the four words
  const uint32_t k = (uint32_t)r >> 6;
  const uint64_t m = sv_lane() == (int)w ? 1ull << (r & 63) : 0ull;
  const int k0 = __builtin_amdgcn_readfirstlane((int)k);
  if (__builtin_amdgcn_ballot_w64((int)k != k0) == 0) {
    switch (k0) {
      case 0: sb.v[0] = set ? (sb.v[0] | m) : (sb.v[0] & ~m); break;
      case 1: sb.v[1] = set ? (sb.v[1] | m) : (sb.v[1] & ~m); break;
      case 2: sb.v[2] = set ? (sb.v[2] | m) : (sb.v[2] & ~m); break;
      default: sb.v[3] = set ? (sb.v[3] | m) : (sb.v[3] & ~m); break;
    }
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint64_t mj = j == k ? m : 0ull;
    sb.v[j] = set ? (sb.v[j] | mj) : (sb.v[j] & ~mj);
  }
}
__device__ __forceinline__ void sbs(WarpSb& sb, uint32_t w, uint8_t r) { sb_upd(sb, w, r, true); }
__device__ __forceinline__ void sbc(WarpSb& sb, uint32_t w, uint8_t r) { sb_upd(sb, w, r, false); }
__device__ __forceinline__ void sbz(WarpSb& sb, uint32_t w) {
  if (sv_lane() == (int)w) sb.v[0] = sb.v[1] = sb.v[2] = sb.v[3] = 0;
}

// (B is SMState, or SmSplit whose members are references: strip those)
#define SV_REF(m) std::remove_reference_t<decltype(B::m)>& m
#define SV_VAL(m) std::remove_reference_t<decltype(B::m)> m
#define SV_WARP(m) WarpReg<std::remove_extent_t<std::remove_reference_t<decltype(B::m)>>> m

template <class B>
struct SmView {
  B& base;
  SV_VAL(id);
  SV_REF(l1_sets);
  SV_REF(l1_assoc);
  SV_REF(cycle);
  SV_VAL(last_progress);
  SV_VAL(epoch_end);
  SV_VAL(out_port_free);
  SV_REF(inj_t0_fs);
  SV_REF(inj_allow0);
  SV_REF(inj_used);
  SV_VAL(age_ctr);
  SV_REF(arb_next);
  SV_REF(arb_cnt);
  SV_WARP(w_next);
  SV_WARP(w_end);
  SV_WARP(w_head);
  SV_WARP(w_age);
  SV_WARP(w_flags);
  SV_WARP(w_ibuf);
  SV_WARP(w_cta);
  SV_WARP(w_inflight);
  SV_WARP(w_stores);
  SV_WARP(w_loads);
  SV_REF(w_wait);
  SV_REF(w_slot_lds);
  SV_REF(w_lds_st);
  WarpSb w_sb;
  SV_REF(w_issue_ok);
  SV_REF(w_win);
  SV_WARP(w_slot_used);
  SV_REF(w_slot_pend);
  SV_REF(w_slot_dst);
  SV_REF(cta_id);
  SV_WARP(cta_valid);
  SV_WARP(cta_live);
  SV_WARP(cta_bar);
  SV_WARP(cta_nexit);
  SV_REF(cta_ks);
  SV_REF(cta_wbase);
  SV_REF(cta_nw);
  SV_REF(n_cta_k);
  SV_REF(cta_wmask);
  SV_REF(used_thr);
  SV_REF(used_regs);
  SV_REF(used_shmem);
  SV_VAL(n_cta_active);
  SV_VAL(n_warps_live);
  SV_VAL(live_mask);
  SV_VAL(n_wait_flags);
  SV_VAL(fetch_rr);
  SV_WARP(sched_last);
  SV_REF(idoc_inst);
  SV_WARP(idoc_meta);
  SV_REF(oc_inst);
  SV_WARP(oc_info);
  SV_WARP(oc_banks);
  SV_WARP(oc_age);
  SV_WARP(fu_next);
  SV_REF(wb_cnt);
  SV_REF(wb);
  SV_VAL(ldst);
  SV_REF(ldst_acc);
  SV_REF(hit_cnt);
  SV_REF(hit);
  SV_REF(l1);
  SV_REF(mshr);
  SV_REF(pend);
  SV_VAL(n_pend);
  SV_REF(il1);
  SV_REF(imshr);
  SV_REF(cl1);
  SV_REF(cmshr);
  SV_WARP(w_iline);
  SV_VAL(idoc_mask);
  SV_VAL(oc_mask);
  SV_VAL(oc_read_mask);
  SV_VAL(l1_stamp);
  SV_WARP(wb_occ);
  SV_WARP(hit_occ);
  SV_VAL(skipped_cycles);
  SV_VAL(min_emit);
  SV_REF(outq);
  SV_VAL(outq_head);
  SV_VAL(outq_n);
  SV_VAL(outstanding);
  SV_REF(ocnt);
  SV_REF(inq);
  SV_VAL(inq_head);
  SV_VAL(inq_n);
  SV_REF(rsp_cl);
  SV_REF(rsp_ld);
  SV_VAL(cl_head);
  SV_VAL(cl_n);
  SV_VAL(ld_head);
  SV_VAL(ld_n);
  SV_REF(skey);
  SV_REF(sref);
  SV_REF(srank);
  // statistics: counter word k lives in lane (k & 63) of word st<k >> 6>, so an
  // update is one masked VALU add instead of an LDS read-modify-write (all
  // words, the per-scheduler issue histograms included: those updates sit
  // in the issue loop, where an LDS round trip each cost ~150 clocks)
  static constexpr int kStv = (kStatWords + 63) / 64;
  static_assert(kStv <= 4, "SmView keeps at most four statistics words per lane");
  // four named words, never an array: a dynamically indexed array (or a
  // merged store through a selected address) demotes the view to scratch
  uint64_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  __device__ __forceinline__ uint64_t stw_get(uint32_t j) const {
    return j == 0 ? st0 : j == 1 ? st1 : j == 2 ? st2 : st3;
  }
  __device__ __forceinline__ void sadd(uint32_t k, uint64_t d) {
    const uint64_t dd = sv_lane() == (int)(k & 63u) ? d : 0ull;
    const uint32_t j = k >> 6;
    st0 += j == 0 ? dd : 0ull;
    if (kStv > 1) st1 += j == 1 ? dd : 0ull;
    if (kStv > 2) st2 += j == 2 ? dd : 0ull;
    if (kStv > 3) st3 += j == 3 ? dd : 0ull;
  }
  // k in [LO, HI) (sm.h SMState::sadd_r): only that range's words are
  // selected, at compile time -- a single-word range is one masked add
  template <uint32_t LO, uint32_t HI>
  __device__ __forceinline__ void sadd_r(uint32_t k, uint64_t d) {
    constexpr uint32_t j0 = LO >> 6, j1 = (HI - 1) >> 6;
    static_assert(LO < HI && j1 < (uint32_t)kStv, "statistics range outside the register words");
    const uint64_t dd = sv_lane() == (int)(k & 63u) ? d : 0ull;
    const uint32_t j = k >> 6;
    if constexpr (j0 <= 0 && 0 <= j1) st0 += (j0 == j1 || j == 0) ? dd : 0ull;
    if constexpr (j0 <= 1 && 1 <= j1) st1 += (j0 == j1 || j == 1) ? dd : 0ull;
    if constexpr (j0 <= 2 && 2 <= j1) st2 += (j0 == j1 || j == 2) ? dd : 0ull;
    if constexpr (j0 <= 3 && 3 <= j1) st3 += (j0 == j1 || j == 3) ? dd : 0ull;
  }
  __device__ __forceinline__ uint64_t sget(uint32_t k) const {
    const uint64_t m = stw_get(k >> 6);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, (int)(k & 63u));
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), (int)(k & 63u));
    return ((uint64_t)hi << 32) | lo;
  }
  __device__ __forceinline__ void sset(uint32_t k, uint64_t v) {
    const bool me = sv_lane() == (int)(k & 63u);
    const uint32_t j = k >> 6;
    st0 = me && j == 0 ? v : st0;
    if (kStv > 1) st1 = me && j == 1 ? v : st1;
    if (kStv > 2) st2 = me && j == 2 ? v : st2;
    if (kStv > 3) st3 = me && j == 3 ? v : st3;
  }

#define SV_SCALARS(X)                                                                                   \
  X(id) X(last_progress) X(epoch_end) X(out_port_free) X(age_ctr) X(n_cta_active)    \
  X(n_warps_live) X(live_mask) X(n_wait_flags) X(fetch_rr) X(n_pend) X(idoc_mask) X(oc_mask) X(oc_read_mask)         \
  X(l1_stamp) X(skipped_cycles) X(min_emit) X(outq_head) X(outq_n) X(outstanding) X(inq_head) X(inq_n) X(cl_head) X(cl_n) X(ld_head) X(ld_n)
#define SV_WARPS(X) \
  X(w_next) X(w_end) X(w_head) X(w_age) X(w_flags) X(w_ibuf) X(w_cta) X(w_inflight) X(w_stores) X(w_loads) X(w_slot_used) \
  X(idoc_meta) X(oc_info) X(oc_banks) X(oc_age) X(fu_next) X(wb_occ) X(hit_occ) X(cta_valid) X(cta_live) X(cta_bar) \
  X(cta_nexit) X(sched_last) X(w_iline)

  __device__ __forceinline__ explicit SmView(B& b)
      : base(b), l1_sets(b.l1_sets), l1_assoc(b.l1_assoc), cycle(b.cycle), inj_t0_fs(b.inj_t0_fs),
        inj_allow0(b.inj_allow0), inj_used(b.inj_used), arb_next(b.arb_next),
        arb_cnt(b.arb_cnt), w_wait(b.w_wait), w_slot_lds(b.w_slot_lds), w_lds_st(b.w_lds_st), w_issue_ok(b.w_issue_ok), w_win(b.w_win),
        w_slot_pend(b.w_slot_pend),
        w_slot_dst(b.w_slot_dst), cta_id(b.cta_id), cta_ks(b.cta_ks), cta_wbase(b.cta_wbase), cta_nw(b.cta_nw),
        n_cta_k(b.n_cta_k), cta_wmask(b.cta_wmask), used_thr(b.used_thr), used_regs(b.used_regs),
        used_shmem(b.used_shmem),
        idoc_inst(b.idoc_inst), oc_inst(b.oc_inst),
        wb_cnt(b.wb_cnt), wb(b.wb), ldst_acc(b.ldst_acc), hit_cnt(b.hit_cnt), hit(b.hit), l1(b.l1), mshr(b.mshr),
        pend(b.pend), il1(b.il1), imshr(b.imshr), cl1(b.cl1), cmshr(b.cmshr),
        outq(b.outq), ocnt(b.ocnt), inq(b.inq), rsp_cl(b.rsp_cl), rsp_ld(b.rsp_ld), skey(b.skey), sref(b.sref), srank(b.srank) {
#define SV_LD(m) m = sv_uni(b.m);
    SV_SCALARS(SV_LD)
#undef SV_LD
#define SV_LDW(m) m.load(b.m);
    SV_WARPS(SV_LDW)
#undef SV_LDW
    w_sb.load(b.w_sb);
    {
      const uint64_t* sw = reinterpret_cast<const uint64_t*>(&b.st);
      const int l = sv_lane();
      auto ld = [&](int j) -> uint64_t { return l + 64 * j < kStatWords ? sw[l + 64 * j < kStatWords ? l + 64 * j : 0] : 0ull; };
      st0 = ld(0);
      if (kStv > 1) st1 = ld(1);
      if (kStv > 2) st2 = ld(2);
      if (kStv > 3) st3 = ld(3);
    }
    {  // LdstState: 16-byte words through readfirstlane
      uint32_t w[sizeof(ldst) / 4];
      __builtin_memcpy(w, &b.ldst, sizeof(ldst));
#pragma unroll
      for (int i = 0; i < (int)(sizeof(ldst) / 4); ++i) w[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)w[i]);
      __builtin_memcpy(&ldst, w, sizeof(ldst));
    }
  }
  // write everything held in registers back to the LDS state
  __device__ __forceinline__ void flush() {
#define SV_ST(m) base.m = m;
    SV_SCALARS(SV_ST)
#undef SV_ST
#define SV_STW(m) m.store(base.m);
    SV_WARPS(SV_STW)
#undef SV_STW
    w_sb.store(base.w_sb);
    {
      uint64_t* sw = reinterpret_cast<uint64_t*>(&base.st);
      const int l = sv_lane();
      if (l < kStatWords) sw[l] = st0;
      if (kStv > 1 && l + 64 < kStatWords) sw[l + 64] = st1;
      if (kStv > 2 && l + 128 < kStatWords) sw[l + 128] = st2;
      if (kStv > 3 && l + 192 < kStatWords) sw[l + 192] = st3;
    }
    base.ldst = ldst;
  }
#undef SV_SCALARS
#undef SV_WARPS
};

#undef SV_REF
#undef SV_VAL
#undef SV_WARP

}  // namespace asim
