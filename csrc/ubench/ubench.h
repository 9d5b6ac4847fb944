// Shared helpers of the CDNA4 (gfx950) micro-benchmark suite.
//
// Counterpart of the reference's util/tuner/GPU_Microbenchmark (hw_def/*.h,
// common/common.mk): every program measures one hardware property of the
// MI355X it runs on and prints it (a) human readable and (b) as
// "-<gpgpusim option> <value>" lines that the tuner
// (accel_sim_framework_distributed_amd/tuner) folds into a gpgpusim.config.
//
// Timing: in-kernel latency chains use s_memtime (shader-clock ticks) in one
// asm statement with its lgkmcnt wait (cdna_hip_programming.md, in-kernel
// stamps); throughput uses hipEvents around back-to-back launches.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#define UB_CHECK(x)                                                                                   \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) {                                                                           \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
      exit(2);                                                                                        \
    }                                                                                                 \
  } while (0)

__device__ __forceinline__ uint64_t ub_clock() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ uint64_t ub_realtime() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

struct UbDevice {
  hipDeviceProp_t p;
  int dev = 0;
  UbDevice() {
    UB_CHECK(hipGetDevice(&dev));
    UB_CHECK(hipGetDeviceProperties(&p, dev));
  }
  int cus() const { return p.multiProcessorCount; }
  double clock_mhz() const { return p.clockRate / 1000.0; }
};

// shader clock (MHz) measured as d(s_memtime) / d(s_memrealtime @ 100 MHz)
__global__ void ub_clock_kernel(uint64_t* out, int spin) {
  uint64_t c0 = ub_clock(), r0 = ub_realtime();
  float x = (float)threadIdx.x;
  for (int i = 0; i < spin; ++i) x = __builtin_fmaf(x, 1.0000001f, 0.5f);
  uint64_t c1 = ub_clock(), r1 = ub_realtime();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = r1 - r0;
    out[2] = (uint64_t)x;
  }
}

inline double ub_shader_mhz() {
  uint64_t* d;
  UB_CHECK(hipMalloc(&d, 3 * sizeof(uint64_t)));
  uint64_t h[3] = {};
  for (int rep = 0; rep < 3; ++rep) {  // warm the clock up
    hipLaunchKernelGGL(ub_clock_kernel, dim3(1), dim3(64), 0, 0, d, 1 << 22);
    UB_CHECK(hipDeviceSynchronize());
  }
  UB_CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  UB_CHECK(hipFree(d));
  return h[1] ? (double)h[0] / (double)h[1] * 100.0 : 0.0;
}

// random cyclic permutation with `n` nodes spaced `stride_elems` apart: the
// pointer-chase visits each node once per lap and defeats prefetching
inline std::vector<uint32_t> ub_chase(size_t n, size_t stride_elems, size_t total_elems, uint32_t seed = 1) {
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0u);
  std::mt19937 g(seed);
  std::shuffle(order.begin() + 1, order.end(), g);
  std::vector<uint32_t> next(total_elems, 0);
  for (size_t i = 0; i < n; ++i) {
    size_t a = order[i] * stride_elems, b = order[(i + 1) % n] * stride_elems;
    next[a] = (uint32_t)b;
  }
  return next;
}

// one lane walks the chain `iters` times; returns average ticks per load
__global__ void ub_chase_kernel(const uint32_t* next, uint32_t start, int warm, int iters, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t j = start;
  // keep the index in a VGPR: a uniform chain could be compiled to scalar
  // (s_load / constant cache) loads, which is not the path being measured
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  for (int i = 0; i < warm; ++i) j = next[j];
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) j = next[j];
  uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = j;
}

inline double ub_chase_latency(size_t bytes, size_t stride_bytes, int iters, bool uncached_warm = false) {
  const size_t total = bytes / 4, stride = std::max<size_t>(1, stride_bytes / 4);
  const size_t n = std::max<size_t>(2, total / stride);
  auto h = ub_chase(n, stride, total);
  uint32_t* d;
  uint64_t* o;
  UB_CHECK(hipMalloc(&d, total * 4));
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMemcpy(d, h.data(), total * 4, hipMemcpyHostToDevice));
  const int warm = uncached_warm ? 0 : (int)std::min<size_t>(n, 1 << 20);
  hipLaunchKernelGGL(ub_chase_kernel, dim3(1), dim3(64), 0, 0, d, 0u, warm, iters, o);
  UB_CHECK(hipDeviceSynchronize());
  uint64_t r[2];
  UB_CHECK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
  UB_CHECK(hipFree(d));
  UB_CHECK(hipFree(o));
  return (double)r[0] / iters;
}

struct UbTimer {
  hipEvent_t a, b;
  UbTimer() {
    UB_CHECK(hipEventCreate(&a));
    UB_CHECK(hipEventCreate(&b));
  }
  ~UbTimer() {
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
  }
  void start() { UB_CHECK(hipEventRecord(a)); }
  float stop_ms() {
    UB_CHECK(hipEventRecord(b));
    UB_CHECK(hipEventSynchronize(b));
    float ms = 0;
    UB_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
  }
};

inline void ub_opt(const char* flag, const std::string& v) { printf("%s %s\n", flag, v.c_str()); }
inline void ub_opt(const char* flag, long long v) { printf("%s %lld\n", flag, v); }
