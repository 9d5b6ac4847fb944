// Global atomic throughput and address conflicts (reference GPU_Microbenchmark
// atomics/Atomic_add_bw, Atomic_add_bw_conflict).  Every CU runs 16 waves of
// global_atomic_add (no return) in three patterns:
//   distinct - every lane its own 128 B line (no two lanes share a line)
//   line     - the 64 lanes of a wave hit 16 words of 4 lines (lane-linear)
//   same     - every lane of every wave adds to one address
// Atomics execute in the L2 (TCC), so the rates are whole-chip operations per
// shader cycle; the conflict cost feeds the notes on -gpgpu_l2_rop_latency
// (ub_atomic_kernel measures the latency itself).
#include "ubench.h"

template <int MODE>
__global__ void __launch_bounds__(1024) atom_bw(uint32_t* buf, int iters) {
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  size_t idx;
  if constexpr (MODE == 0) idx = (size_t)gtid * 32;  // one line per lane
  else if constexpr (MODE == 1) idx = (size_t)gtid;  // lane-linear words
  else idx = 0;
  for (int i = 0; i < iters; ++i) __hip_atomic_fetch_add(buf + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
static double run(const char* name, int cus, uint32_t* buf, double mhz) {
  const int threads = 1024, iters = MODE == 2 ? 16 : 256;
  hipLaunchKernelGGL((atom_bw<MODE>), dim3(cus), dim3(threads), 0, 0, buf, 4);
  UB_CHECK(hipDeviceSynchronize());
  UbTimer t;
  t.start();
  hipLaunchKernelGGL((atom_bw<MODE>), dim3(cus), dim3(threads), 0, 0, buf, iters);
  const double ms = t.stop_ms();
  const double ops = (double)cus * threads * iters;
  const double per_clk = ops / (ms * 1e-3 * mhz * 1e6);
  printf("%-8s %10.3f ms  %8.2f Gatomics/s  %8.2f lane-atomics per shader cycle (chip)\n", name, ms,
         ops / (ms * 1e6), per_clk);
  return per_clk;
}

int main() {
  UbDevice dev;
  const double mhz = ub_shader_mhz();
  printf("device %s, %d CUs, %.0f MHz\n", dev.p.gcnArchName, dev.cus(), mhz);
  const size_t n = (size_t)dev.cus() * 1024 * 32 + 64;
  uint32_t* buf;
  UB_CHECK(hipMalloc(&buf, n * 4));
  UB_CHECK(hipMemset(buf, 0, n * 4));
  const double d = run<0>("distinct", dev.cus(), buf, mhz);
  const double l = run<1>("line", dev.cus(), buf, mhz);
  const double s = run<2>("same", dev.cus(), buf, mhz);
  printf("# atomics_per_clk_distinct_lines %.2f\n# atomics_per_clk_lane_linear %.2f\n# atomics_per_clk_same_address %.3f\n",
         d, l, s);
  printf("# same_address_slowdown %.1f\n", s > 0 ? d / s : 0.0);
  UB_CHECK(hipFree(buf));
  return 0;
}
