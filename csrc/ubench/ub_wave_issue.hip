// Issue rate of ONE wave (no reference counterpart; it sets
// -gpgpu_warp_issue_interval): a workgroup of W waves on one CU runs chains of
// 8 independent v_fma_f32 per lane (no dependency stalls at the measured
// 8-cycle latency), each wave timing its own loop with s_memtime.  With one
// wave per SIMD the cycles per instruction are the wave's own issue
// interval; with several waves per SIMD they approach the SIMD's throughput
// (ub_alu's issue interval).  Prints cycles per instruction per wave for
// 1..8 waves per SIMD and the -gpgpu_warp_issue_interval line.
#include "ubench.h"

__global__ void ub_issue_kernel(float m, float c, int iters, uint64_t* out, float* sink) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = (float)(threadIdx.x + k);
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __builtin_fmaf(a[k], m, c);
  }
  const uint64_t t1 = ub_clock();
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  if (s == -12345.f) sink[0] = s;
  if ((threadIdx.x & 63) == 0) out[threadIdx.x / 64] = t1 - t0;
}

int main() {
  UbDevice d;
  const int iters = 4096;
  uint64_t* o;
  float* sink;
  UB_CHECK(hipMalloc(&o, 64 * sizeof(uint64_t)));
  UB_CHECK(hipMalloc(&sink, 64));
  double one_per_simd = 0;
  for (int waves : {1, 4, 8, 16, 32}) {
    hipLaunchKernelGGL(ub_issue_kernel, dim3(1), dim3(64 * waves), 0, 0, 1.0001f, 0.5f, iters, o, sink);
    UB_CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(ub_issue_kernel, dim3(1), dim3(64 * waves), 0, 0, 1.0001f, 0.5f, iters, o, sink);
    UB_CHECK(hipDeviceSynchronize());
    std::vector<uint64_t> h(waves);
    UB_CHECK(hipMemcpy(h.data(), o, waves * sizeof(uint64_t), hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    const double cpi = (double)h[waves / 2] / (iters * 8.0);
    const double per_simd = cpi / std::max(1, waves / 4);
    printf("%2d waves on one CU: %6.2f cycles per FMA instruction per wave (%5.2f per SIMD)\n", waves, cpi,
           waves >= 4 ? per_simd : cpi);
    if (waves == 4) one_per_simd = cpi;
  }
  printf("# wave_issue_cycles %.2f\n", one_per_simd);
  ub_opt("-gpgpu_warp_issue_interval", (long long)std::max(1.0, std::floor(one_per_simd + 0.25)));
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
  return 0;
}
