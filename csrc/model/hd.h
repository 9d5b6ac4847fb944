// Single-source host/device attributes and the "lane policy" abstraction.
//
// The cycle model (csrc/model/*.h) is written ONCE.  Every per-warp /
// per-thread / per-way loop that is embarrassingly parallel is expressed
// through a lane policy `P`:
//   * SeqPar  (this file)        - CPU reference engine: a plain loop.
//   * WavePar (engine/wave_par.h) - GPU engine: one CDNA4 wavefront, lane i
//                                   handles element i (64-wide ballots,
//                                   cross-lane reductions via DPP/shuffles).
// Everything outside those calls is wave-uniform scalar code that every lane
// executes identically on the GPU, so the CPU and GPU engines produce
// bit-identical simulator state.  This replaces the reference's serial STL
// walks (e.g. scheduler_unit::cycle, shader.cc:1249-1556; the coalescer,
// abstract_hardware_model.cc:284-748) with lane-parallel formulations.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define SIM_HD __host__ __device__
#define SIM_HDI __host__ __device__ __forceinline__
// out of line on the device: cold code whose registers must not weigh on the
// engine kernel's hot loops
#define SIM_HDN __host__ __device__ inline __attribute__((noinline))
#else
#define SIM_HDN inline
#define SIM_HD
#define SIM_HDI inline
#endif

namespace asim {

SIM_HDI int popc64(uint64_t x) { return __builtin_popcountll(x); }
SIM_HDI int ffs64(uint64_t x) { return x ? __builtin_ctzll(x) : -1; }
SIM_HDI uint64_t rotr64(uint64_t x, unsigned r, unsigned n) {
  // rotate the low n bits of x right by r (n <= 64, r < n)
  if (r == 0) return x;
  uint64_t m = (n == 64) ? ~0ull : ((1ull << n) - 1);
  x &= m;
  return ((x >> r) | (x << (n - r))) & m;
}
template <class T>
SIM_HDI T amin(T a, T b) { return a < b ? a : b; }
template <class T>
SIM_HDI T amax(T a, T b) { return a > b ? a : b; }

// Sequential lane policy (CPU reference engine).
struct SeqPar {
  static constexpr int kLanes = 64;
  // bit i of the result = f(i) for i < n (n <= 64)
  template <class F>
  static SIM_HDI uint64_t ballot(int n, F&& f) {
    uint64_t m = 0;
    for (int i = 0; i < n; ++i)
      if (f(i)) m |= 1ull << i;
    return m;
  }
  // one pass over n elements split across lanes (here: all of them), then
  // reductions of the per-lane partials (here: identity)
  template <class F>
  static SIM_HDI void lane_loop(int n, F&& f) {
    for (int i = 0; i < n; ++i) f(i);
  }
  static SIM_HDI uint32_t red_sum(uint32_t v) { return v; }
  static SIM_HDI uint32_t red_or(uint32_t v) { return v; }
  static SIM_HDI uint64_t red_sum64(uint64_t v) { return v; }
  static SIM_HDI uint64_t red_min64(uint64_t v) { return v; }
  static SIM_HDI uint64_t red_max64(uint64_t v) { return v; }
  // ballot restricted to the lanes of `mask` (bit i = f(i) && mask bit i):
  // the CPU engine visits only those lanes (e.g. the live warps)
  template <class F>
  static SIM_HDI uint64_t ballot_m(uint64_t mask, F&& f) {
    uint64_t m = 0;
    for (uint64_t r = mask; r; r &= r - 1) {
      const int i = __builtin_ctzll(r);
      if (f(i)) m |= 1ull << i;
    }
    return m;
  }
  template <class F>
  static SIM_HDI void each_m(uint64_t mask, F&& f) {
    for (uint64_t r = mask; r; r &= r - 1) f(__builtin_ctzll(r));
  }
  // run f(i) for every i < n (independent iterations only)
  template <class F>
  static SIM_HDI void each(int n, F&& f) {
    for (int i = 0; i < n; ++i) f(i);
  }
  // side effect executed once per wave (global-memory stores of uniform data)
  template <class F>
  static SIM_HDI void one(F&& f) { f(); }
  // copy n trace records (instructions / access records, 16-byte multiples,
  // at most 1 KB) from the kernel trace into the unit's state.  The GPU policy
  // issues them as asynchronous LDS DMA and the reader calls fetch_wait()
  // first; here it is a plain copy.
  template <class T>
  static SIM_HDI void fetch_copy(T* dst, const T* src, int n) {
    for (int i = 0; i < n; ++i) dst[i] = src[i];
  }
  static SIM_HDI void fetch_wait() {}
  static SIM_HDI void sync() {}
  // stage profiling stamp (no-op on the CPU; the GPU profiling build records
  // s_memtime deltas per stage)
  static SIM_HDI void prof(int) {}
  static SIM_HDI void tick(int) {}
  // wave-uniform value hint (identity here; readfirstlane on the GPU so that
  // the compiler keeps the value and everything derived from it in SGPRs)
  template <class T>
  static SIM_HDI T uni(T v) { return v; }
  // run f on the SM state for an epoch's cycle loop (the GPU policy hands f
  // a register-resident view of the same state, csrc/engine/sm_view.h)
  template <class S, class F>
  static SIM_HDI void view(S& s, F&& f) { f(s); }
  // index i < n minimising key(i) (ties -> lowest i); key == ~0ull means
  // "not a candidate".  Returns -1 if there is no candidate.
  template <class F>
  static SIM_HDI int argmin(int n, F&& key) {
    uint64_t best = ~0ull;
    int bi = -1;
    for (int i = 0; i < n; ++i) {
      uint64_t k = key(i);
      if (k != ~0ull && (bi < 0 || k < best)) {
        best = k;
        bi = i;
      }
    }
    return bi;
  }
  // smallest i < n with pred(i), -1 if none (the argmin of "key = i if
  // candidate" searches: MSHR / free-slot lookups)
  template <class F>
  static SIM_HDI int find_first(int n, F&& pred) {
    for (int i = 0; i < n; ++i)
      if (pred(i)) return i;
    return -1;
  }
  template <class F>
  static SIM_HDI uint32_t sum(int n, F&& f) {
    uint32_t s = 0;
    for (int i = 0; i < n; ++i) s += f(i);
    return s;
  }
  template <class F>
  static SIM_HDI uint32_t vmax(int n, F&& f) {
    uint32_t s = 0;
    for (int i = 0; i < n; ++i) {
      uint32_t v = f(i);
      s = v > s ? v : s;
    }
    return s;
  }
  // per-lane values: lanes<T>(n, f) evaluates f(i) for the lanes i < n; the
  // result gives a lane's own value back (self(i) inside lane-parallel code)
  // and any one lane's value to wave-uniform code (at(i)).  On the CPU it is a
  // lazy re-evaluation; on the GPU a register per lane read by v_readlane.
  template <class T, class F>
  struct Lanes {
    F f;
    SIM_HDI T self(int i) const { return f(i); }
    SIM_HDI T at(int i) const { return f(i); }
  };
  template <class T, class F>
  static SIM_HDI Lanes<T, F> lanes(int, F f) {
    return Lanes<T, F>{f};
  }
  // exclusive prefix sum: out(i, sum_{j<i} val(j)); returns the total
  template <class F, class G>
  static SIM_HDI uint32_t scan(int n, F&& val, G&& out) {
    uint32_t acc = 0;
    for (int i = 0; i < n; ++i) {
      uint32_t v = val(i);
      out(i, acc);
      acc += v;
    }
    return acc;
  }
  template <class F>
  static SIM_HDI uint64_t vor(int n, F&& f) {
    uint64_t s = 0;
    for (int i = 0; i < n; ++i) s |= f(i);
    return s;
  }
  // the members of `mask` (indices < n <= 16) sorted by key ascending (ties
  // to the lower index), packed 4 bits per entry: entry r = (ord >> 4r) & 15.
  // Replaces repeated "oldest remaining" argmin scans with one ranking.
  template <class F>
  static SIM_HDI uint64_t order16(int n, uint32_t mask, F&& key) {
    uint64_t ord = 0;
    for (int i = 0; i < n; ++i) {
      if (!(mask >> i & 1u)) continue;
      const uint32_t ki = key(i);
      uint32_t r = 0;
      for (int j = 0; j < n; ++j)
        if ((mask >> j & 1u) && j != i) {
          const uint32_t kj = key(j);
          r += (kj < ki || (kj == ki && j < i)) ? 1u : 0u;
        }
      ord |= (uint64_t)i << (4 * r);
    }
    return ord;
  }
};

}  // namespace asim
