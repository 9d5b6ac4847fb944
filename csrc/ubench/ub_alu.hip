// Functional-unit latency and initiation interval (reference
// GPU_Microbenchmark core/lat_{float,double,int32}, sfu_lat_fsqrt,
// MaxFlops_*): a dependent chain gives latency, 8 independent chains per
// lane at full occupancy give the issue interval per wavefront.  Prints the
// -trace_opcode_latency_initiation_{sp,dp,int,sfu} lines ("latency,ii").
#include "ubench.h"

template <int OP, class T>
__device__ __forceinline__ T step(T x, T y) {
  if constexpr (OP == 0) return __builtin_fmaf(x, y, (T)0.5f);           // v_fma_f32
  else if constexpr (OP == 1) return __builtin_fma(x, y, (T)0.5);        // v_fma_f64
  else if constexpr (OP == 2) return x * y + (T)7;                       // v_mad_u32_u24 / v_mul_lo+add
  else return __builtin_sqrtf(x + y);                                     // v_sqrt_f32 (transcendental)
}

// y is a kernel argument so the compiler cannot fold the chain into a
// closed form (x * 1 + 7 repeated would become one multiply-add)
template <int OP, class T>
__global__ void lat_kernel(T seed, T y, int iters, uint64_t* out, T* sink) {
  T x = seed + (T)threadIdx.x;
  uint64_t t0 = ub_clock();
#pragma unroll 16
  for (int i = 0; i < iters; ++i) x = step<OP, T>(x, y);
  uint64_t t1 = ub_clock();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (x == (T)-1) sink[0] = x;
}

template <int OP, class T>
__global__ void thr_kernel(T seed, T y, int iters, uint64_t* out, T* sink) {
  T x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = seed + (T)(threadIdx.x + k);
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = step<OP, T>(x[k], y);
  }
  uint64_t t1 = ub_clock();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
  T s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  if (s == (T)-1) sink[0] = s;
}

template <int OP, class T>
static void measure(const char* name, const char* flag, T seed, T y) {
  uint64_t* o;
  T* sink;
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 16));
  const int iters = 1 << 14;
  uint64_t h = 0;
  hipLaunchKernelGGL((lat_kernel<OP, T>), dim3(1), dim3(64), 0, 0, seed, y, iters, o, sink);
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double lat = (double)h / iters;
  // one CU, 4 SIMDs x 4 waves: cycles per wave-instruction per SIMD
  const int waves_per_simd = 4, simds = 4;
  hipLaunchKernelGGL((thr_kernel<OP, T>), dim3(1), dim3(64 * waves_per_simd * simds), 0, 0, seed, y, iters / 4,
                     o, sink);
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double per_inst = (double)h / ((iters / 4) * 8.0 * waves_per_simd);
  printf("%-6s latency %6.2f cycles, issue interval %5.2f cycles/wave-inst per SIMD\n", name, lat, per_inst);
  char v[64];
  snprintf(v, sizeof(v), "%d,%d", (int)(lat + 0.5), std::max(1, (int)(per_inst + 0.5)));
  ub_opt(flag, v);
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
}

// scalar ALU (the CU's scalar unit): a dependent s_add_u32 chain of one wave
__global__ void salu_lat_kernel(uint32_t seed, uint32_t y, int iters, uint64_t* out, uint32_t* sink) {
  uint32_t x = seed;
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; i += 16) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("s_add_u32 %0, %0, %1" : "+s"(x) : "s"(y) : "scc");
  }
  uint64_t t1 = ub_clock();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (x == 0xdeadbeefu) sink[0] = x;
}

static void measure_salu() {
  uint64_t* o;
  uint32_t* sink;
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 16));
  const int iters = 1 << 14;
  uint64_t h = 0;
  hipLaunchKernelGGL(salu_lat_kernel, dim3(1), dim3(64), 0, 0, 3u, 1664525u, iters, o, sink);
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double lat = (double)h / iters;
  printf("%-6s latency %6.2f cycles (dependent chain, one wave)\n", "salu", lat);
  char v[64];
  const int l = std::max(1, (int)(lat + 0.5));
  snprintf(v, sizeof(v), "%d,%d", l, 1);
  ub_opt("-trace_opcode_latency_initiation_spec_op_8", v);
  snprintf(v, sizeof(v), "1,4,%d,4,4,SALU", l);
  ub_opt("-specialized_unit_8", v);
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
}

int main() {
  UbDevice d;
  measure_salu();
  measure<0, float>("fp32", "-trace_opcode_latency_initiation_sp", 1.0001f, 0.9999f);
  measure<1, double>("fp64", "-trace_opcode_latency_initiation_dp", 1.0001, 0.9999);
  measure<2, uint32_t>("int32", "-trace_opcode_latency_initiation_int", 3u, 1664525u);
  measure<3, float>("sqrt", "-trace_opcode_latency_initiation_sfu", 2.0f, 1.0f);
  return 0;
}
