// Instruction-cache capacity and sequential fetch cost (reference
// GPU_Microbenchmark has no icache program; gpgpu-sim's -gpgpu_cache:il1 is
// tuned by hand): one wave runs a straight-line block of K v_add_f32 twice.
// The first pass fetches every code line from L2 (cold), the second runs
// from the instruction cache while the block fits in it.  Cold cycles per
// instruction close to warm ones mean the sequential prefetcher hides the
// line fetches; the block size where warm time rises is the capacity.
#include "ubench.h"

#define A1 "v_add_f32 %0, 1.0, %0\n"
#define A8 A1 A1 A1 A1 A1 A1 A1 A1
#define A64 A8 A8 A8 A8 A8 A8 A8 A8

template <int N>
__device__ __forceinline__ void body(float& x) {
  asm volatile(A64 : "+v"(x));
  if constexpr (N > 1) body<N - 1>(x);
}

template <int N>
__global__ void k_code(float* sink, uint64_t* out) {
  float x = threadIdx.x;
  for (int r = 0; r < 2; ++r) {
    const uint64_t t0 = ub_clock();
    body<N>(x);
    const uint64_t t1 = ub_clock();
    if (threadIdx.x == 0) out[r] = t1 - t0;
  }
  if (x == -1.f) sink[0] = x;
}

template <int N>
static void run(float* sink, uint64_t* o, double* cold, double* warm) {
  hipLaunchKernelGGL(k_code<N>, dim3(1), dim3(64), 0, 0, sink, o);
  uint64_t h[2];
  UB_CHECK(hipMemcpy(h, o, 16, hipMemcpyDeviceToHost));
  const double n = 64.0 * N;
  *cold = h[0] / n;
  *warm = h[1] / n;
  printf("code %6d B (%5d insts): cold %6.2f  warm %6.2f cycles/inst\n", N * 64 * 4, N * 64, *cold, *warm);
}

int main() {
  UbDevice d;
  float* sink;
  uint64_t* o;
  UB_CHECK(hipMalloc(&sink, 16));
  UB_CHECK(hipMalloc(&o, 16));
  double c[6], w[6];
  run<8>(sink, o, &c[0], &w[0]);     //   2 KB
  run<32>(sink, o, &c[1], &w[1]);    //   8 KB
  run<64>(sink, o, &c[2], &w[2]);    //  16 KB
  run<128>(sink, o, &c[3], &w[3]);   //  32 KB
  run<256>(sink, o, &c[4], &w[4]);   //  64 KB
  run<512>(sink, o, &c[5], &w[5]);   // 128 KB
  const int sizes[6] = {2, 8, 16, 32, 64, 128};
  int cap = 0;
  for (int i = 1; i < 6; ++i)
    if (w[i] > 1.25 * w[0]) {
      cap = sizes[i - 1];
      break;
    }
  // cold fetch cost beyond the warm issue cost, per 128-byte line (32 insts)
  const double per_line = (c[3] - w[3]) * 32.0;
  printf("# cold_extra_cycles_per_line %.1f\n", per_line);
  // a fetch that is fully hidden costs nothing extra per line; an exposed
  // L2 fetch costs ~its latency: the prefetch depth that hides it
  const int pf = per_line < 20 ? 8 : per_line < 60 ? 4 : per_line < 150 ? 2 : 0;
  ub_opt("-gpgpu_inst_prefetch_lines", pf);
  if (cap) {
    printf("# icache_kb %d\n", cap);
    char v[96];
    snprintf(v, sizeof(v), "N:%d:128:4,L:R:f:N:L,S:4:64,4", std::max(1, cap * 1024 / 128 / 4));
    ub_opt("-gpgpu_cache:il1", v);
  } else {
    // straight-line code re-run from L2 at the warm rate: the prefetcher hides
    // capacity misses too, so the capacity is not observable this way
    printf("# icache capacity not resolved (sequential prefetch hides capacity misses up to 128 KB)\n");
  }
  UB_CHECK(hipFree(sink));
  UB_CHECK(hipFree(o));
  return 0;
}
