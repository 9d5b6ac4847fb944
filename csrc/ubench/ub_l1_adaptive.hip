// Does the vector L1 give up capacity to LDS?  (reference GPU_Microbenchmark
// l1_cache/l1_adaptive: on Volta/Ampere L1 and shared memory share one
// array and the driver's carve-out changes the L1 size.)  One lane
// pointer-chases footprints of 8..64 KB in a kernel that also holds 0, 64 or
// 160 KB of LDS; if the L1 knee (the footprint where the latency leaves the
// L1 hit level) does not move with the LDS allocation, L1 and LDS are
// separate arrays and the simulator must not carve one out of the other:
// -gpgpu_adaptive_cache_config 0.
#include "ubench.h"

__global__ void __launch_bounds__(64) chase_lds(const uint32_t* next, int warm, int iters, uint64_t* out) {
  extern __shared__ uint32_t lds[];
  if (threadIdx.x != 0) return;
  lds[0] = 1;  // the allocation is real (the dynamic size sets occupancy)
  uint32_t j = 0;
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  for (int i = 0; i < warm; ++i) j = next[j];
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) j = next[j];
  const uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = j + lds[0];
}

int main() {
  UbDevice dev;
  const size_t lds_max = std::max(dev.p.sharedMemPerBlock, dev.p.sharedMemPerBlockOptin);
  printf("device %s, LDS per workgroup max %zu KB\n", dev.p.gcnArchName, lds_max / 1024);
  const size_t kb[] = {8, 16, 24, 28, 32, 40, 48, 64};
  const size_t lds_kb[] = {0, 64, 160};
  uint64_t* o;
  UB_CHECK(hipMalloc(&o, 16));
  double knee[3] = {};
  double lat[3][8] = {};
  for (int li = 0; li < 3; ++li) {
    const size_t lb = std::min<size_t>(lds_kb[li] * 1024, lds_max);
    if (lb > 64 * 1024) UB_CHECK(hipFuncSetAttribute((const void*)chase_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb));
    for (int i = 0; i < 8; ++i) {
      const size_t bytes = kb[i] * 1024, stride = 32;  // 128 B: one node per line
      const size_t total = bytes / 4, n = total / stride;
      auto h = ub_chase(n, stride, total, 5);
      uint32_t* d;
      UB_CHECK(hipMalloc(&d, total * 4));
      UB_CHECK(hipMemcpy(d, h.data(), total * 4, hipMemcpyHostToDevice));
      const int iters = 4096;
      hipLaunchKernelGGL(chase_lds, dim3(1), dim3(64), lb, 0, d, (int)n * 2, iters, o);
      UB_CHECK(hipDeviceSynchronize());
      uint64_t r[2];
      UB_CHECK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
      lat[li][i] = (double)r[0] / iters;
      UB_CHECK(hipFree(d));
    }
    const double hit = lat[li][0];
    for (int i = 0; i < 8; ++i)
      if (lat[li][i] > 1.5 * hit) {
        knee[li] = (double)kb[i];
        break;
      }
    printf("LDS %3zu KB:", lb / 1024);
    for (int i = 0; i < 8; ++i) printf(" %zuK=%.0f", kb[i], lat[li][i]);
    printf("  (first footprint past the L1: %.0f KB)\n", knee[li]);
  }
  const bool fixed = knee[0] == knee[1] && knee[1] == knee[2];
  printf("# l1_knee_kb_lds0 %.0f\n# l1_knee_kb_lds64 %.0f\n# l1_knee_kb_lds160 %.0f\n# l1_shares_array_with_lds %d\n",
         knee[0], knee[1], knee[2], fixed ? 0 : 1);
  ub_opt("-gpgpu_adaptive_cache_config", fixed ? 0 : 1);
  UB_CHECK(hipFree(o));
  return 0;
}
