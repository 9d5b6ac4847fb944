// Does a kernel launch start with a cold instruction cache?  (no reference
// counterpart: GPGPU-Sim keeps the L1I across kernels.)  The same kernel --
// ~6 KB of straight-line code, four workgroups per CU so that every CU's SQC
// has run it -- is launched four times back to back, synchronised; under
//   rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -- ub_icache_launch
// every dispatch's misses are counted (hw_stats/icache_launch.py).  Equal
// misses on every launch: the dispatch invalidates the SQC
// (-sim_sqc_invalidate_at_launch 1); misses on the first launch only: the
// cache keeps the code (0).
#include "ubench.h"

#define BODY4(x) x = __builtin_fmaf(x, 1.0001f, 0.5f); x = __builtin_fmaf(x, 0.9999f, 0.25f); \
                 x = __builtin_fmaf(x, 1.0002f, 0.125f); x = __builtin_fmaf(x, 0.9998f, 0.0625f);
#define BODY16(x) BODY4(x) BODY4(x) BODY4(x) BODY4(x)
#define BODY64(x) BODY16(x) BODY16(x) BODY16(x) BODY16(x)
#define BODY256(x) BODY64(x) BODY64(x) BODY64(x) BODY64(x)

__global__ void __launch_bounds__(64) icl_kernel(float* out, float seed) {
  float x = seed + (float)threadIdx.x;
  BODY256(x)
  BODY256(x)
  BODY256(x)
  if (x == -1.f) out[threadIdx.x] = x;
}

int main() {
  UbDevice d;
  printf("device %s, %d CUs\n", d.p.gcnArchName, d.cus());
  float* out;
  UB_CHECK(hipMalloc(&out, 256));
  for (int r = 0; r < 4; ++r) {
    hipLaunchKernelGGL(icl_kernel, dim3(d.cus() * 4), dim3(64), 0, 0, out, 1.0f);
    UB_CHECK(hipDeviceSynchronize());
  }
  printf("icache launch: 4 launches done\n");
  UB_CHECK(hipFree(out));
  return 0;
}
