// Matrix-core (MFMA) latency and throughput on gfx950 (reference
// GPU_Microbenchmark core/tensor_lat_half, tensor_bw_half with WMMA):
// v_mfma_f32_32x32x16_bf16 dependent-accumulator chain for latency, four
// independent accumulators per wave on every SIMD of every CU for the chip's
// dense bf16 rate.  Prints -trace_opcode_latency_initiation_tensor.
#include "ubench.h"

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;

__global__ void mfma_lat(int iters, uint64_t* out, float* sink) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)0.5f;
  }
  f32x16 c = {};
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  uint64_t t1 = ub_clock();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c[i];
  if (s == -1.f) sink[0] = s;
}

__global__ void mfma_thr(int iters, uint64_t* out, float* sink) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)0.5f;
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  uint64_t t1 = ub_clock();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  if (s == -1.f) sink[0] = s;
}

int main() {
  UbDevice d;
  uint64_t* o;
  float* sink;
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 16));
  const int iters = 4096;
  uint64_t h = 0;
  hipLaunchKernelGGL(mfma_lat, dim3(1), dim3(64), 0, 0, iters, o, sink);
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double lat = (double)h / iters;
  // per-SIMD issue interval: 4 waves per CU (one per SIMD), 4 chains each
  hipLaunchKernelGGL(mfma_thr, dim3(1), dim3(256), 0, 0, iters, o, sink);
  UB_CHECK(hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost));
  const double ii = (double)h / (iters * 4.0);
  // whole chip, timed with events
  const int cus = d.cus();
  UbTimer t;
  hipLaunchKernelGGL(mfma_thr, dim3(cus * 4), dim3(256), 0, 0, iters, o, sink);
  UB_CHECK(hipDeviceSynchronize());
  t.start();
  hipLaunchKernelGGL(mfma_thr, dim3(cus * 4), dim3(256), 0, 0, iters, o, sink);
  const float ms = t.stop_ms();
  const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (cus * 4 * 4);  // per wave: 4 chains
  printf("mfma_f32_32x32x16_bf16: dependent latency %.1f cycles, issue interval %.1f cycles/SIMD, chip %.1f TFLOP/s\n",
         lat, ii, flops / (ms * 1e-3) / 1e12);
  char v[64];
  snprintf(v, sizeof(v), "%d,%d", (int)(lat + 0.5), std::max(1, (int)(ii + 0.5)));
  ub_opt("-trace_opcode_latency_initiation_tensor", v);
  printf("# mfma_bf16_tflops %.1f\n", flops / (ms * 1e-3) / 1e12);
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
  return 0;
}
