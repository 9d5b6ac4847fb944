// CDNA4 wavefront lane policy: one 64-lane wavefront executes the model of
// one SM (or one memory channel).  Lane i handles element i of every
// lane-parallel section; reductions use cross-lane shuffles (DPP/ds_swizzle
// lowering) and 64-bit ballots.  Uniform code outside these calls runs
// redundantly on all lanes against LDS-resident state.
#pragma once
#include <hip/hip_runtime.h>

#include "../model/hd.h"
#include "sm_view.h"

namespace asim {

struct WavePar {
  static constexpr int kLanes = 64;
  static __device__ __forceinline__ int lane() { return (int)(threadIdx.x & 63); }

  template <class F>
  static __device__ __forceinline__ uint64_t ballot(int n, F&& f) {
    const int l = lane();
    bool p = false;
    if (l < n) p = f(l);
    return (uint64_t)__ballot(p);
  }
  template <class F>
  static __device__ __forceinline__ void lane_loop(int n, F&& f) {
    for (int i = lane(); i < n; i += 64) f(i);
  }
  static __device__ __forceinline__ uint32_t red_sum(uint32_t v) {
    return wave_reduce(v, [](uint32_t a, uint32_t b) { return a + b; });
  }
  static __device__ __forceinline__ uint32_t red_or(uint32_t v) {
    return wave_reduce(v, [](uint32_t a, uint32_t b) { return a | b; });
  }
  static __device__ __forceinline__ uint64_t red_sum64(uint64_t v) {
    // lane partials of 64-bit sums: reduce the two halves as 32-bit sums of
    // 16-bit limbs so no carry is lost (64 lanes x 2^16 fits in 32 bits)
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t limb = (uint32_t)(v >> (16 * k)) & 0xffffu;
      r += (uint64_t)wave_reduce(limb, [](uint32_t a, uint32_t b) { return a + b; }) << (16 * k);
    }
    return r;
  }
  template <bool kMax>
  static __device__ __forceinline__ uint64_t red64(uint64_t v) {
    uint32_t h = (uint32_t)(v >> 32), l = (uint32_t)v;
    auto step = [&](uint32_t oh, uint32_t ol) {
      const bool take = kMax ? (oh > h || (oh == h && ol > l)) : (oh < h || (oh == h && ol < l));
      if (take) { h = oh; l = ol; }
    };
    step(dpp<0xB1>(h), dpp<0xB1>(l));
    step(dpp<0x4E>(h), dpp<0x4E>(l));
    step(dpp<0x141>(h), dpp<0x141>(l));
    step(dpp<0x140>(h), dpp<0x140>(l));
    uint32_t rh = rdl(h, 0), rl = rdl(l, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
      const uint32_t oh = rdl(h, r), ol = rdl(l, r);
      const bool take = kMax ? (oh > rh || (oh == rh && ol > rl)) : (oh < rh || (oh == rh && ol < rl));
      if (take) { rh = oh; rl = ol; }
    }
    return ((uint64_t)rh << 32) | rl;
  }
  static __device__ __forceinline__ uint64_t red_min64(uint64_t v) { return red64<false>(v); }
  static __device__ __forceinline__ uint64_t red_max64(uint64_t v) { return red64<true>(v); }
  template <class F>
  static __device__ __forceinline__ uint64_t ballot_m(uint64_t mask, F&& f) {
    const int l = lane();
    bool p = false;
    if ((mask >> l) & 1ull) p = f(l);
    return (uint64_t)__ballot(p);
  }
  template <class F>
  static __device__ __forceinline__ void each_m(uint64_t mask, F&& f) {
    const int l = lane();
    if ((mask >> l) & 1ull) f(l);
  }
  template <class F>
  static __device__ __forceinline__ void each(int n, F&& f) {
    for (int i = lane(); i < n; i += 64) f(i);
  }
  template <class F>
  static __device__ __forceinline__ void one(F&& f) {
    if (lane() == 0) f();
  }
  // trace records HBM -> LDS without VGPR staging: lane i moves 16 bytes
  // (global_load_lds, lane-linear LDS image at a wave-uniform base); the
  // copy completes asynchronously, fetch_wait() is the reader's wait
  template <class T>
  static __device__ __forceinline__ void fetch_copy(T* dst, const T* src, int n) {
    static_assert(sizeof(T) % 16 == 0, "fetch_copy: 16-byte granular records");
    typedef __attribute__((address_space(1))) const uint4 g4;
    typedef __attribute__((address_space(3))) uint4 l4;
    const int chunks = n * (int)(sizeof(T) / 16);
    const int l = lane();
    if (l >= chunks) return;
    // a unit simulated in place in HBM (the global-state engine build): a
    // plain vector copy (fetch_wait's vmcnt wait covers its stores too)
    typedef __attribute__((address_space(0))) const void flat_cv;
    if (!__builtin_amdgcn_is_shared((flat_cv*)dst)) {
      reinterpret_cast<uint4*>(dst)[l] = reinterpret_cast<const uint4*>(src)[l];
      return;
    }
    __builtin_amdgcn_global_load_lds((g4*)(reinterpret_cast<const uint4*>(src) + l), (l4*)dst, 16, 0, 0);
  }
  static __device__ __forceinline__ void fetch_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
  static __device__ __forceinline__ void prof(int) {}
  static __device__ __forceinline__ void tick(int) {}
  // Values read from LDS state land in VGPRs (the compiler cannot know that
  // every lane read the same word), so all arithmetic and control flow
  // derived from them runs as 64-lane VALU code with exec masking.
  // readfirstlane makes the value -- and what is computed from it -- scalar.
  template <class T>
  static __device__ __forceinline__ T uni(T v) {
    static_assert(sizeof(T) <= 4 || sizeof(T) % 4 == 0, "uni: 1/2/4-byte or word-multiple types");
    static_assert(std::is_trivially_copyable<T>::value, "uni: values only (cast proxies first)");
    if constexpr (sizeof(T) <= 4) {
      uint32_t u = 0;
      __builtin_memcpy(&u, &v, sizeof(T));
      u = (uint32_t)__builtin_amdgcn_readfirstlane((int)u);
      T r;
      __builtin_memcpy(&r, &u, sizeof(T));
      return r;
    } else {
      uint32_t w[sizeof(T) / 4];
      __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
      for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)w[i]);
      T r;
      __builtin_memcpy(&r, w, sizeof(T));
      return r;
    }
  }

  static __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // the cycle loop runs on a register-resident view of the LDS state
  template <class S, class F>
  static __device__ __forceinline__ void view(S& s, F&& f) {
    sync();
    SmView<S> v(s);
    f(v);
    v.flush();
    sync();
  }
  // ---- cross-lane reductions on DPP row operations (no LDS traffic) ----
  // Every reduction runs in wave-uniform control flow with all 64 lanes
  // active.  Within a 16-lane row: quad_perm xor 1 / xor 2, row_half_mirror,
  // row_mirror (each a register-to-register v_mov_dpp); across the 4 rows:
  // v_readlane into SGPRs.  A __shfl_xor reduction compiles to ds_bpermute,
  // an LDS round trip per step (~6 dependent LDS latencies per reduction).
  template <int Ctrl>
  static __device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, Ctrl, 0xf, 0xf, false);
  }
  static __device__ __forceinline__ uint32_t rdl(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
  }
  template <class Op>
  static __device__ __forceinline__ uint32_t row_reduce(uint32_t v, Op op) {
    v = op(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp<0x141>(v));  // row_half_mirror
    v = op(v, dpp<0x140>(v));  // row_mirror
    return v;
  }
  template <class Op>
  static __device__ __forceinline__ uint32_t wave_reduce(uint32_t v, Op op) {
    v = row_reduce(v, op);
    return op(op(rdl(v, 0), rdl(v, 16)), op(rdl(v, 32), rdl(v, 48)));
  }
  // (key, index) pair: smaller key wins, ties to the smaller index
  static __device__ __forceinline__ bool kless(uint32_t ah, uint32_t al, uint32_t ai, uint32_t bh, uint32_t bl,
                                               uint32_t bi) {
    return ah < bh || (ah == bh && (al < bl || (al == bl && ai < bi)));
  }
  template <int Ctrl>
  static __device__ __forceinline__ void kstep(uint32_t& h, uint32_t& l, uint32_t& i) {
    const uint32_t oh = dpp<Ctrl>(h), ol = dpp<Ctrl>(l), oi = dpp<Ctrl>(i);
    if (kless(oh, ol, oi, h, l, i)) {
      h = oh;
      l = ol;
      i = oi;
    }
  }
  template <class F>
  static __device__ __forceinline__ int argmin(int n, F&& key) {
    uint64_t best = ~0ull;
    uint32_t bi = 0x7fffffffu;
    for (int i = lane(); i < n; i += 64) {
      uint64_t k = key(i);
      if (k != ~0ull && (k < best || (k == best && (uint32_t)i < bi))) {
        best = k;
        bi = (uint32_t)i;
      }
    }
    uint32_t h = (uint32_t)(best >> 32), l = (uint32_t)best;
    kstep<0xB1>(h, l, bi);
    kstep<0x4E>(h, l, bi);
    kstep<0x141>(h, l, bi);
    kstep<0x140>(h, l, bi);
    uint32_t rh = rdl(h, 0), rl = rdl(l, 0), ri = rdl(bi, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
      const uint32_t oh = rdl(h, r), ol = rdl(l, r), oi = rdl(bi, r);
      if (kless(oh, ol, oi, rh, rl, ri)) {
        rh = oh;
        rl = ol;
        ri = oi;
      }
    }
    return (rh == ~0u && rl == ~0u) ? -1 : (int)ri;
  }
  // per-lane values (hd.h SeqPar::lanes): computed once per lane, handed to
  // uniform code with one v_readlane per 32-bit word
  template <class T>
  struct LaneVal {
    T v;
    __device__ __forceinline__ T self(int) const { return v; }
    __device__ __forceinline__ T at(int i) const {
      static_assert(sizeof(T) % 4 == 0, "LaneVal: word-multiple types");
      uint32_t w[sizeof(T) / 4];
      __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
      for (int k = 0; k < (int)(sizeof(T) / 4); ++k) w[k] = rdl(w[k], i);
      T r;
      __builtin_memcpy(&r, w, sizeof(T));
      return r;
    }
  };
  template <class T, class F>
  static __device__ __forceinline__ LaneVal<T> lanes(int n, F&& f) {
    LaneVal<T> r;
    if (lane() < n) r.v = f(lane());
    else __builtin_memset(&r.v, 0, sizeof(T));
    return r;
  }
  // members of `mask` (n <= 16) by ascending key, 4 bits per rank (hd.h
  // SeqPar::order16): lane i ranks itself against every member (readlane
  // loop over the mask in SGPRs), then one OR-reduction packs the order
  template <class F>
  static __device__ __forceinline__ uint64_t order16(int n, uint32_t mask, F&& key) {
    const int l = lane();
    const bool mine = l < n && (mask >> l & 1u);
    const uint32_t k = mine ? (uint32_t)key(l) : 0u;
    uint32_t r = 0;
    for (uint32_t m = mask; m;) {
      const int j = __builtin_ctz(m);
      m &= m - 1;
      const uint32_t kj = rdl(k, j);
      r += (j != l && (kj < k || (kj == k && j < l))) ? 1u : 0u;
    }
    const uint64_t v = mine ? ((uint64_t)(uint32_t)l << (4 * r)) : 0ull;
    auto o = [](uint32_t a, uint32_t b) { return a | b; };
    const uint32_t lo = wave_reduce((uint32_t)v, o), hi = wave_reduce((uint32_t)(v >> 32), o);
    return ((uint64_t)hi << 32) | lo;
  }
  // smallest i < n with pred(i): four 64-lane chunks are evaluated (their
  // loads in flight together) before the first hit is picked by ballot + ffs
  template <class F>
  static __device__ __forceinline__ int find_first(int n, F&& pred) {
    const int l = lane();
    for (int b = 0; b < n; b += 256) {
      bool p0 = false, p1 = false, p2 = false, p3 = false;
      if (b + l < n) p0 = pred(b + l);
      if (b + 64 < n && b + 64 + l < n) p1 = pred(b + 64 + l);
      if (b + 128 < n && b + 128 + l < n) p2 = pred(b + 128 + l);
      if (b + 192 < n && b + 192 + l < n) p3 = pred(b + 192 + l);
      const uint64_t m0 = (uint64_t)__ballot(p0), m1 = (uint64_t)__ballot(p1), m2 = (uint64_t)__ballot(p2),
                     m3 = (uint64_t)__ballot(p3);
      if (m0) return b + __builtin_ctzll(m0);
      if (m1) return b + 64 + __builtin_ctzll(m1);
      if (m2) return b + 128 + __builtin_ctzll(m2);
      if (m3) return b + 192 + __builtin_ctzll(m3);
    }
    return -1;
  }
  template <class F>
  static __device__ __forceinline__ uint32_t sum(int n, F&& f) {
    uint32_t s = 0;
    for (int i = lane(); i < n; i += 64) s += f(i);
    return wave_reduce(s, [](uint32_t a, uint32_t b) { return a + b; });
  }
  template <class F>
  static __device__ __forceinline__ uint32_t vmax(int n, F&& f) {
    uint32_t s = 0;
    for (int i = lane(); i < n; i += 64) {
      uint32_t v = f(i);
      s = v > s ? v : s;
    }
    return wave_reduce(s, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
  }
  template <class F>
  static __device__ __forceinline__ uint64_t vor(int n, F&& f) {
    uint64_t s = 0;
    for (int i = lane(); i < n; i += 64) s |= f(i);
    auto o = [](uint32_t a, uint32_t b) { return a | b; };
    const uint32_t lo = wave_reduce((uint32_t)s, o), hi = wave_reduce((uint32_t)(s >> 32), o);
    return ((uint64_t)hi << 32) | lo;
  }
  // exclusive scan: within-row Hillis-Steele on row_shr:1/2/4/8 (lanes
  // shifted in from outside the row read 0), then the row totals via readlane
  template <class F, class G>
  static __device__ __forceinline__ uint32_t scan(int n, F&& val, G&& out) {
    uint32_t carry = 0;
    const int l = lane();
    for (int b = 0; b < n; b += 64) {
      const int i = b + l;
      uint32_t v = i < n ? val(i) : 0u;
      uint32_t inc = v;
      inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x111, 0xf, 0xf, false);  // row_shr:1
      inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x112, 0xf, 0xf, false);  // row_shr:2
      inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x114, 0xf, 0xf, false);  // row_shr:4
      inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x118, 0xf, 0xf, false);  // row_shr:8
      const uint32_t t0 = rdl(inc, 15), t1 = rdl(inc, 31), t2 = rdl(inc, 47), t3 = rdl(inc, 63);
      const int row = l >> 4;
      inc += row == 0 ? 0u : row == 1 ? t0 : row == 2 ? t0 + t1 : t0 + t1 + t2;
      if (i < n) out(i, carry + inc - v);
      carry += t0 + t1 + t2 + t3;
    }
    return carry;
  }
};

}  // namespace asim
