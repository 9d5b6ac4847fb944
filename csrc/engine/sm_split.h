// Split state of one simulated SM for the MI355X engine's split-state build
// (ASIM_GPU_STATE=split): the SMState fields before SMState::wb_cnt (the hot
// part: warps, pipeline registers, collectors, queues, statistics, ~32 KB)
// live in the block's LDS, the geometry-sized arrays from wb_cnt on
// (writeback and hit rings, L1 / instruction / constant cache tags, MSHRs,
// the pending-load table, ~86 KB) stay in the unit's HBM image.  SmSplit
// re-exposes every SMState member under its own name as a reference into one
// or the other, so the single-source model (csrc/model, templated on the
// state type) runs unchanged on it, and the register view (sm_view.h) builds
// on it like on SMState.  A block then needs ~35 KB of LDS: four engine
// waves share a CU where the LDS-state build fits one.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace asim {

// the hot prefix (LDS) ends where the tail begins (16-byte aligned: the
// copies in and out of LDS move whole 16-byte words)
constexpr size_t kSmHotBytes = offsetof(SMState, wb_cnt);
static_assert(kSmHotBytes % 16 == 0, "SMState::wb_cnt must start a 16-byte word");
static_assert(offsetof(SMState, st) + sizeof(SMStats) <= kSmHotBytes, "statistics belong to the hot part");

#define ASIM_SM_FIELDS(X) \
  X(id) X(l1_sets) X(l1_assoc) X(cycle) X(last_progress) X(epoch_end) X(out_port_free) X(inj_t0_fs) \
  X(inj_allow0) X(inj_used) X(age_ctr) X(arb_next) X(arb_cnt) X(w_next) X(w_end) X(w_head) \
  X(w_age) X(w_flags) X(w_ibuf) X(w_cta) X(w_inflight) X(w_stores) X(w_loads) X(w_wait) \
  X(w_sb) X(w_issue_ok) X(w_win) X(w_slot_used) X(w_slot_lds) X(w_lds_st) X(w_pad) X(w_slot_pend) \
  X(w_slot_dst) X(cta_id) X(cta_valid) X(cta_live) X(cta_bar) X(cta_nexit) X(cta_ks) X(cta_wbase) \
  X(cta_nw) X(n_cta_k) X(cta_wmask) X(used_thr) X(used_regs) X(used_shmem) X(n_cta_active) X(n_warps_live) \
  X(live_mask) X(n_wait_flags) X(fetch_rr) X(sched_last) X(idoc_inst) X(idoc_meta) X(oc_inst) X(oc_info) \
  X(oc_banks) X(oc_age) X(fu_next) X(ldst) X(ldst_acc) X(n_pend) X(w_iline) X(idoc_mask) \
  X(oc_mask) X(oc_read_mask) X(l1_stamp) X(wb_occ) X(hit_occ) X(skipped_cycles) X(min_emit) X(outq) \
  X(outq_head) X(outq_n) X(outstanding) X(pub_nz) X(ocnt) X(inq) X(inq_head) X(inq_n) \
  X(rsp_cl) X(rsp_ld) X(cl_head) X(cl_n) X(ld_head) X(ld_n) X(skey) X(sref) \
  X(srank) X(k_uid) X(next_cta) X(next_ctax) X(st) X(wb_cnt) X(wb) X(hit_cnt) \
  X(hit) X(l1) X(mshr) X(pend) X(il1) X(imshr) X(cl1) X(cmshr)

struct SmSplit {
#define SS_DECL(m) decltype(SMState::m)& m;
  ASIM_SM_FIELDS(SS_DECL)
#undef SS_DECL
  // hot: the LDS copy of the prefix; cold: the unit's HBM image
  __device__ __forceinline__ SmSplit(SMState& hot, SMState& cold)
      :
#define SS_INIT(m) m(*(offsetof(SMState, m) < kSmHotBytes ? &hot.m : &cold.m)),
        ASIM_SM_FIELDS(SS_INIT) pad_(0) {
  }
#undef SS_INIT
  int pad_;
  __device__ __forceinline__ void sadd(uint32_t k, uint64_t d) { reinterpret_cast<uint64_t*>(&st)[k] += d; }
  __device__ __forceinline__ uint64_t sget(uint32_t k) const { return reinterpret_cast<const uint64_t*>(&st)[k]; }
  __device__ __forceinline__ void sset(uint32_t k, uint64_t v) { reinterpret_cast<uint64_t*>(&st)[k] = v; }
  template <uint32_t LO, uint32_t HI>
  __device__ __forceinline__ void sadd_r(uint32_t k, uint64_t d) {
    sadd(k, d);
  }
};

}  // namespace asim
