// CDNA4 wavefront lane policy: one 64-lane wavefront executes the model of
// one SM (or one memory channel).  Lane i handles element i of every
// lane-parallel section; reductions use cross-lane shuffles (DPP/ds_swizzle
// lowering) and 64-bit ballots.  Uniform code outside these calls runs
// redundantly on all lanes against LDS-resident state.
#pragma once
#include <hip/hip_runtime.h>

#include "../model/hd.h"

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
  static __device__ __forceinline__ void each(int n, F&& f) {
    for (int i = lane(); i < n; i += 64) f(i);
  }
  template <class F>
  static __device__ __forceinline__ void one(F&& f) {
    if (lane() == 0) f();
  }
  static __device__ __forceinline__ void prof(int) {}
  static __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  static __device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_xor(lo, m, 64);
    hi = __shfl_xor(hi, m, 64);
    return ((uint64_t)hi << 32) | lo;
  }
  template <class F>
  static __device__ __forceinline__ int argmin(int n, F&& key) {
    uint64_t best = ~0ull;
    int bi = 0x7fffffff;
    for (int i = lane(); i < n; i += 64) {
      uint64_t k = key(i);
      if (k != ~0ull && (k < best || (k == best && i < bi))) {
        best = k;
        bi = i;
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      uint64_t ob = shfl_xor64(best, m);
      int oi = __shfl_xor(bi, m, 64);
      if (ob < best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    return best == ~0ull ? -1 : bi;
  }
  template <class F>
  static __device__ __forceinline__ uint32_t sum(int n, F&& f) {
    uint32_t s = 0;
    for (int i = lane(); i < n; i += 64) s += f(i);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    return s;
  }
  template <class F>
  static __device__ __forceinline__ uint32_t vmax(int n, F&& f) {
    uint32_t s = 0;
    for (int i = lane(); i < n; i += 64) {
      uint32_t v = f(i);
      s = v > s ? v : s;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      uint32_t o = __shfl_xor(s, m, 64);
      s = o > s ? o : s;
    }
    return s;
  }
  template <class F>
  static __device__ __forceinline__ uint64_t vor(int n, F&& f) {
    uint64_t s = 0;
    for (int i = lane(); i < n; i += 64) s |= f(i);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s |= shfl_xor64(s, m);
    return s;
  }
  template <class F, class G>
  static __device__ __forceinline__ uint32_t scan(int n, F&& val, G&& out) {
    uint32_t carry = 0;
    const int l = lane();
    for (int b = 0; b < n; b += 64) {
      const int i = b + l;
      uint32_t v = i < n ? val(i) : 0u;
      uint32_t inc = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(inc, d, 64);
        if (l >= d) inc += o;
      }
      if (i < n) out(i, carry + inc - v);
      carry += __shfl(inc, 63, 64);
    }
    return carry;
  }
};

}  // namespace asim
