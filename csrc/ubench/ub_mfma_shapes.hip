// Matrix-core latency and throughput per MFMA shape and type on gfx950
// (reference GPU_Microbenchmark core/tensor_lat_{half,float,...} and
// tensor_bw_*): a dependent-accumulator chain gives latency, four
// independent accumulators per wave at one wave per SIMD the issue interval;
// FLOP/cycle/CU from the throughput.  The bf16 32x32x16 row is the tensor
// pipe the CDNA traces use (-trace_opcode_latency_initiation_tensor).
#include "ubench.h"

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(8 * sizeof(_Float16)))) _Float16 f16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;
typedef __attribute__((__vector_size__(16 * sizeof(int)))) int i32x16;
typedef __attribute__((__vector_size__(4 * sizeof(int)))) int i32x4;

template <int S, class C>
__device__ __forceinline__ C step(C c) {
  if constexpr (S == 0) { bf16x8 a; for (int i = 0; i < 8; ++i) a[i] = (__bf16)0.5f; return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c, 0, 0, 0); }
  else if constexpr (S == 1) { bf16x8 a; for (int i = 0; i < 8; ++i) a[i] = (__bf16)0.5f; return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c, 0, 0, 0); }
  else if constexpr (S == 2) { f16x8 a; for (int i = 0; i < 8; ++i) a[i] = (_Float16)0.5f; return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, a, c, 0, 0, 0); }
  else if constexpr (S == 3) return __builtin_amdgcn_mfma_f32_32x32x2f32(0.5f, 0.25f, c, 0, 0, 0);
  else if constexpr (S == 4) return __builtin_amdgcn_mfma_f32_16x16x4f32(0.5f, 0.25f, c, 0, 0, 0);
  else { i32x4 a = {1, 1, 1, 1}; return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c, 0, 0, 0); }
}

template <int S, class C>
__global__ void k_lat(int iters, uint64_t* out, float* sink) {
  C c = {};
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) c = step<S, C>(c);
  const uint64_t t1 = ub_clock();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if ((float)c[0] == -1.f) sink[0] = 1.f;
}

template <int S, class C>
__global__ void k_thr(int iters, uint64_t* out, float* sink) {
  C c0 = {}, c1 = {}, c2 = {}, c3 = {};
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
    c0 = step<S, C>(c0);
    c1 = step<S, C>(c1);
    c2 = step<S, C>(c2);
    c3 = step<S, C>(c3);
  }
  const uint64_t t1 = ub_clock();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
  if ((float)(c0[0] + c1[0] + c2[0] + c3[0]) == -1.f) sink[0] = 1.f;
}

template <int S, class C>
static void measure(const char* name, double flops, uint64_t* o, float* sink, bool tuner) {
  const int iters = 2048;
  uint64_t h = 0;
  hipLaunchKernelGGL((k_lat<S, C>), dim3(1), dim3(64), 0, 0, iters, o, sink);
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double lat = (double)h / iters;
  hipLaunchKernelGGL((k_thr<S, C>), dim3(1), dim3(256), 0, 0, iters, o, sink);  // one wave per SIMD
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double ii = (double)h / (iters * 4.0);
  printf("%-22s latency %6.1f  issue interval %6.1f cycles/SIMD  %7.0f FLOP/cycle/CU\n", name, lat, ii,
         4.0 * flops / ii);
  if (tuner) {
    char v[64];
    snprintf(v, sizeof(v), "%d,%d", (int)(lat + 0.5), std::max(1, (int)(ii + 0.5)));
    ub_opt("-trace_opcode_latency_initiation_tensor", v);
  }
}

int main() {
  UbDevice d;
  uint64_t* o;
  float* sink;
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 16));
  measure<0, f32x16>("mfma_f32_32x32x16_bf16", 2.0 * 32 * 32 * 16, o, sink, true);
  measure<1, f32x4>("mfma_f32_16x16x32_bf16", 2.0 * 16 * 16 * 32, o, sink, false);
  measure<2, f32x16>("mfma_f32_32x32x16_f16", 2.0 * 32 * 32 * 16, o, sink, false);
  measure<3, f32x16>("mfma_f32_32x32x2_f32", 2.0 * 32 * 32 * 2 * 2, o, sink, false);
  measure<4, f32x4>("mfma_f32_16x16x4_f32", 2.0 * 16 * 16 * 4 * 4, o, sink, false);
  measure<5, i32x16>("mfma_i32_32x32x32_i8", 2.0 * 32 * 32 * 32, o, sink, false);
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
  return 0;
}
