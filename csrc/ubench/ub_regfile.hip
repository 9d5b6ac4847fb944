// VGPR operand bandwidth (reference GPU_Microbenchmark core/regfile_bw):
// does a three-source VALU op slow down when its sources sit in the same
// register bank?  Eight independent v_fma_f32 chains per lane at 16 waves per
// CU; in one variant the three sources of each fma are registers with equal
// index mod 4 (one bank of a 4-bank file), in the other they differ mod 4.
// Equal issue intervals mean operand reads are not bank limited at this
// rate; the simulator's operand collector then needs enough banks for no
// conflicts to appear: -gpgpu_num_reg_banks is printed as a suggestion.
#include "ubench.h"

template <bool SAME>
__global__ void __launch_bounds__(1024) rf(int iters, uint64_t* out, float* sink) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
    if constexpr (SAME) {
      // v4 = fma(v4, v8, v12): all sources index = 0 mod 4
      asm volatile(
          "v_fma_f32 v4, v4, v8, v12\n\tv_fma_f32 v5, v5, v9, v13\n\tv_fma_f32 v6, v6, v10, v14\n\t"
          "v_fma_f32 v7, v7, v11, v15\n\tv_fma_f32 v16, v16, v20, v24\n\tv_fma_f32 v17, v17, v21, v25\n\t"
          "v_fma_f32 v18, v18, v22, v26\n\tv_fma_f32 v19, v19, v23, v27" ::
              : "v4", "v5", "v6", "v7", "v16", "v17", "v18", "v19");
    } else {
      asm volatile(
          "v_fma_f32 v4, v4, v9, v14\n\tv_fma_f32 v5, v5, v10, v15\n\tv_fma_f32 v6, v6, v11, v12\n\t"
          "v_fma_f32 v7, v7, v8, v13\n\tv_fma_f32 v16, v16, v21, v26\n\tv_fma_f32 v17, v17, v22, v27\n\t"
          "v_fma_f32 v18, v18, v23, v24\n\tv_fma_f32 v19, v19, v20, v25" ::
              : "v4", "v5", "v6", "v7", "v16", "v17", "v18", "v19");
    }
  }
  const uint64_t t1 = ub_clock();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
  const float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (s == -1.f) sink[0] = s;
}

template <bool SAME>
static double run(uint64_t* o, float* sink) {
  const int iters = 1 << 14, threads = 1024;  // 16 waves: 4 per SIMD
  hipLaunchKernelGGL((rf<SAME>), dim3(1), dim3(threads), 0, 0, 64, o, sink);
  hipLaunchKernelGGL((rf<SAME>), dim3(1), dim3(threads), 0, 0, iters, o, sink);
  UB_CHECK(hipDeviceSynchronize());
  uint64_t c = 0;
  UB_CHECK(hipMemcpy(&c, o, 8, hipMemcpyDeviceToHost));
  return (double)c / (iters * 8.0 * 4);  // cycles per wave-instruction per SIMD
}

int main() {
  UbDevice dev;
  printf("device %s\n", dev.p.gcnArchName);
  uint64_t* o;
  float* sink;
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 16));
  const double same = run<true>(o, sink), diff = run<false>(o, sink);
  printf("v_fma_f32 issue interval: sources in one bank %.3f, spread over banks %.3f cycles/wave-inst per SIMD\n",
         same, diff);
  const bool conflict = same > 1.1 * diff;
  printf("# vgpr_same_bank_interval %.3f\n# vgpr_spread_bank_interval %.3f\n# vgpr_bank_conflicts_visible %d\n", same,
         diff, conflict ? 1 : 0);
  printf("# suggest_gpgpu_num_reg_banks %d\n", conflict ? 4 : 16);
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
  return 0;
}
