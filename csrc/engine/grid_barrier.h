// Grid-wide barrier of the persistent engine kernel (and of the
// ub_grid_barrier micro-benchmark that prices it).  Every block must be
// co-resident; blocks are grouped by blockIdx % 8 (a speed hint for XCD
// locality, correctness does not depend on placement).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace asim {

struct GpuCtl {  // zeroed by hipMemsetAsync before every launch
  uint32_t arrive[8][64];     // per-group arrival counters (one 256-B line each)
  uint32_t gen[8][64];        // per-group generation words: each group polls its own line
  uint32_t top[64];           // group leaders' counter
  uint32_t error;             // barrier timeout / fault code
  uint32_t done;
  uint32_t deadlock;
  uint32_t cap;  // a run cap (-gpgpu_max_insn / _max_cta / _max_completed_cta) ended the launch
  uint64_t end_cycle;
  uint64_t end_epoch;
  uint64_t epochs_run;
};

// grid barrier: blocks are grouped by blockIdx % 8 (which shares an XCD under
// the observed round-robin placement: a speed hint only, correctness does not
// depend on it).  Monotonic counters; the last arriver of a group forwards to
// the top counter, the last group leader bumps every group's generation word,
// and each block polls only its own group's word (relaxed, with s_sleep), so
// no single line is hammered by every block while the arrivals queue behind
// it.  One agent release before arriving and one agent acquire after leaving.
// `b`: the block's index among the `nblocks` that synchronise (blockIdx.x
// for a whole launch; a batch launch's simulation numbers its own blocks)
template <bool kFence = true>
__device__ __forceinline__ bool grid_barrier_b(GpuCtl* ctl, uint32_t b, uint32_t nblocks, uint32_t epoch_in_launch,
                                               uint32_t* was_last = nullptr) {
  const uint32_t grp = b & 7u;
  const uint32_t ngrp = nblocks < 8 ? nblocks : 8u;
  const uint32_t in_grp = (nblocks - grp + 7u) / 8u;  // members of this group
  const uint32_t target = epoch_in_launch + 1u;
  bool ok = true;
  uint32_t last = 0;
  // every lane's stores must be complete and visible at agent scope
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (kFence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) {
    uint32_t prev = __hip_atomic_fetch_add(&ctl->arrive[grp][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1u == target * in_grp) {
      // last of its group: forward to the top counter
      uint32_t t = __hip_atomic_fetch_add(&ctl->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1u == target * ngrp) last = 1;
      if (t + 1u == target * ngrp)
        for (uint32_t g = 0; g < ngrp; ++g)
          __hip_atomic_store(&ctl->gen[g][0], target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t spins = 0;
    while (__hip_atomic_load(&ctl->gen[grp][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1ull << 25)) {  // ~seconds: give up, report, let every block exit
        __hip_atomic_store(&ctl->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
      if ((spins & 15) == 0 && __hip_atomic_load(&ctl->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        ok = false;
        break;
      }
    }
  }
  ok = __builtin_amdgcn_readlane(ok ? 1 : 0, 0) != 0;
  if (was_last) *was_last = (uint32_t)__builtin_amdgcn_readlane((int)last, 0);
  if (kFence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return ok;
}
template <bool kFence = true>
__device__ __forceinline__ bool grid_barrier(GpuCtl* ctl, uint32_t nblocks, uint32_t epoch_in_launch,
                                             uint32_t* was_last = nullptr) {
  return grid_barrier_b<kFence>(ctl, blockIdx.x, nblocks, epoch_in_launch, was_last);
}

}  // namespace asim
