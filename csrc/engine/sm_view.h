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
    if (__builtin_amdgcn_ballot_w64(w != w0) == 0)
      return (T)__builtin_amdgcn_readlane((int)(uint32_t)v, w0);
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
  template <class A>
  __device__ __forceinline__ void load(const A& arr) {
    v = arr[sv_lane()];
  }
  template <class A>
  __device__ __forceinline__ void store(A& arr) const {
    arr[sv_lane()] = v;
  }
};

#define SV_REF(m) decltype(B::m)& m
#define SV_VAL(m) decltype(B::m) m
#define SV_WARP(m) WarpReg<typename std::remove_extent<decltype(B::m)>::type> m

// statistics: scalars in registers, arrays by reference
template <class B>
struct SmStatsView {
  SV_VAL(thread_insn);
  SV_VAL(warp_insn);
  SV_REF(cls_insn);
  SV_VAL(active_cycles);
  SV_VAL(busy_cycles);
  SV_VAL(issue_stall_idle);
  SV_VAL(sb_stall);
  SV_VAL(pipe_stall);
  SV_REF(l1);
  SV_VAL(shmem_acc);
  SV_VAL(shmem_conflict_cycles);
  SV_VAL(pkts_out);
  SV_VAL(pkts_in);
  SV_VAL(bytes_out);
  SV_VAL(bytes_in);
  SV_VAL(rf_reads);
  SV_VAL(rf_writes);
  SV_VAL(oc_bank_conflicts);
  SV_VAL(ctas_done);
  SV_VAL(warps_done);
  SV_VAL(occupancy_acc);
  SV_VAL(mem_insn);
  SV_REF(power_acc);
  SV_VAL(mf_lat_sum);
  SV_VAL(mf_lat_n);
  SV_VAL(mf_lat_max);
  SV_REF(mf_lat_hist);
  SV_REF(il1);
#define SV_SCALARS(X)                                                                                    \
  X(thread_insn) X(warp_insn) X(active_cycles) X(busy_cycles) X(issue_stall_idle) X(sb_stall) X(pipe_stall) \
  X(shmem_acc) X(shmem_conflict_cycles) X(pkts_out) X(pkts_in) X(bytes_out) X(bytes_in) X(rf_reads)         \
  X(rf_writes) X(oc_bank_conflicts) X(ctas_done) X(warps_done) X(occupancy_acc) X(mem_insn) X(mf_lat_sum)   \
  X(mf_lat_n) X(mf_lat_max)
  __device__ __forceinline__ explicit SmStatsView(B& b)
      : cls_insn(b.cls_insn), l1(b.l1), power_acc(b.power_acc), mf_lat_hist(b.mf_lat_hist), il1(b.il1) {
#define SV_LD(m) m = sv_uni(b.m);
    SV_SCALARS(SV_LD)
#undef SV_LD
  }
  __device__ __forceinline__ void flush(B& b) const {
#define SV_ST(m) b.m = m;
    SV_SCALARS(SV_ST)
#undef SV_ST
  }
#undef SV_SCALARS
};

template <class B>
struct SmView {
  B& base;
  SV_VAL(id);
  SV_VAL(kernel_cta_slots);
  SV_REF(cycle);
  SV_VAL(last_progress);
  SV_VAL(epoch_end);
  SV_VAL(out_port_free);
  SV_VAL(age_ctr);
  SV_WARP(w_next);
  SV_WARP(w_end);
  SV_WARP(w_head);
  SV_REF(w_wfill);
  SV_WARP(w_age);
  SV_WARP(w_flags);
  SV_WARP(w_ibuf);
  SV_WARP(w_cta);
  SV_WARP(w_inflight);
  SV_WARP(w_stores);
  SV_WARP(w_loads);
  SV_REF(w_sb);
  SV_WARP(w_slot_used);
  SV_REF(w_slot_pend);
  SV_REF(w_slot_dst);
  SV_REF(w_win);
  SV_REF(cta_id);
  SV_REF(cta_valid);
  SV_REF(cta_live);
  SV_REF(cta_bar);
  SV_REF(cta_nexit);
  SV_VAL(n_cta_active);
  SV_VAL(n_warps_live);
  SV_VAL(n_wait_flags);
  SV_VAL(fetch_rr);
  SV_REF(sched_last);
  SV_REF(idoc);
  SV_REF(oc);
  SV_REF(fu_next);
  SV_REF(wb_cnt);
  SV_REF(wb);
  SV_VAL(ldst);
  SV_REF(hit_cnt);
  SV_REF(hit);
  SV_REF(l1);
  SV_REF(mshr);
  SV_REF(pend);
  SV_VAL(n_pend);
  SV_REF(il1);
  SV_REF(imshr);
  SV_REF(w_iline);
  SV_VAL(idoc_mask);
  SV_VAL(oc_mask);
  SV_VAL(oc_read_mask);
  SV_VAL(l1_stamp);
  SV_REF(wb_occ);
  SV_REF(hit_occ);
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
  SV_REF(skey);
  SV_REF(sref);
  SV_REF(srank);
  SV_REF(ks);
  decltype(B::st)& st;  // statistics stay in LDS (SGPR pressure)

#define SV_SCALARS(X)                                                                                   \
  X(id) X(kernel_cta_slots) X(last_progress) X(epoch_end) X(out_port_free) X(age_ctr) X(n_cta_active)    \
  X(n_warps_live) X(n_wait_flags) X(fetch_rr) X(n_pend) X(idoc_mask) X(oc_mask) X(oc_read_mask)         \
  X(l1_stamp) X(skipped_cycles) X(min_emit) X(outq_head) X(outq_n) X(outstanding) X(inq_head) X(inq_n)
#define SV_WARPS(X) \
  X(w_next) X(w_end) X(w_head) X(w_age) X(w_flags) X(w_ibuf) X(w_cta) X(w_inflight) X(w_stores) X(w_loads) X(w_slot_used)

  __device__ __forceinline__ explicit SmView(B& b)
      : base(b), cycle(b.cycle), w_wfill(b.w_wfill), w_sb(b.w_sb), w_slot_pend(b.w_slot_pend),
        w_slot_dst(b.w_slot_dst), w_win(b.w_win), cta_id(b.cta_id), cta_valid(b.cta_valid), cta_live(b.cta_live),
        cta_bar(b.cta_bar), cta_nexit(b.cta_nexit), sched_last(b.sched_last), idoc(b.idoc), oc(b.oc),
        fu_next(b.fu_next), wb_cnt(b.wb_cnt), wb(b.wb), hit_cnt(b.hit_cnt), hit(b.hit), l1(b.l1), mshr(b.mshr),
        pend(b.pend), il1(b.il1), imshr(b.imshr), w_iline(b.w_iline), wb_occ(b.wb_occ), hit_occ(b.hit_occ),
        outq(b.outq), ocnt(b.ocnt), inq(b.inq), skey(b.skey), sref(b.sref), srank(b.srank), ks(b.ks), st(b.st) {
#define SV_LD(m) m = sv_uni(b.m);
    SV_SCALARS(SV_LD)
#undef SV_LD
#define SV_LDW(m) m.load(b.m);
    SV_WARPS(SV_LDW)
#undef SV_LDW
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
    base.ldst = ldst;
  }
#undef SV_SCALARS
#undef SV_WARPS
};

#undef SV_REF
#undef SV_VAL
#undef SV_WARP

}  // namespace asim
