// Cache access granularity and memory-level parallelism of one CU (reference
// GPU_Microbenchmark l1_cache/l1_sector, l2_cache/l2_stride_cons,
// mem/mem_stride_cons and l1_cache/l1_mshr), measured on the gfx950 it runs on.
//
// 1. Granularity: one wave issues K independent 64-lane loads, lane i reading
//    base + i * stride; the wave's footprint is 64 * stride bytes.  The time
//    per wave-load grows with the number of distinct lines (or sectors) the
//    wave touches, so the stride where the cost starts to double is the
//    granule: for an L2-resident buffer the L2 -> L1 fill granule, for a
//    footprint far beyond the last-level cache the HBM request granule.
// 2. Memory-level parallelism: one lane walks P independent pointer chains
//    through an HBM-sized buffer, interleaved.  While the misses overlap, the
//    time per round stays at one miss latency; past the number of misses the
//    CU can keep in flight it grows linearly.  Printed raw (relative round
//    time per chain count): chains 4 KB apart also measure channel / TLB
//    effects, so no MSHR count is derived from them automatically.
#include "ubench.h"

__global__ void __launch_bounds__(64) gran_kernel(const float* __restrict__ a, size_t stride_f, int k, size_t mask_f,
                                                  size_t base_f, int warm, uint64_t* out, float* sink) {
  const int l = threadIdx.x;
  float acc = 0.f;
  // warm pass over the same addresses (L2-resident runs); none for HBM runs
  if (warm)
    for (int r = 0; r < k; ++r) acc += a[(base_f + (size_t)r * 64 * stride_f + l * stride_f) & mask_f];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t t0 = ub_clock();
#pragma unroll 8
  for (int r = 0; r < k; ++r) acc += a[(base_f + (size_t)r * 64 * stride_f + l * stride_f) & mask_f];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t t1 = ub_clock();
  if (l == 0) out[0] = t1 - t0;
  if (acc == -1.f) sink[0] = acc;
}

__global__ void __launch_bounds__(64) mlp_kernel(const uint32_t* __restrict__ next, int chains, int rounds,
                                                 uint32_t stride, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t p[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) p[c] = (uint32_t)c * stride;
  asm volatile("" ::: "memory");
  const uint64_t t0 = ub_clock();
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int c = 0; c < 32; ++c)
      if (c < chains) p[c] = next[p[c]];
  }
  const uint64_t t1 = ub_clock();
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < 32; ++c) x ^= p[c];
  out[0] = t1 - t0;
  out[1] = x;
}

int main() {
  UbDevice dev;
  printf("device %s, %d CUs\n", dev.p.gcnArchName, dev.cus());
  uint64_t* d_out;
  float* sink;
  UB_CHECK(hipMalloc(&d_out, 16));
  UB_CHECK(hipMalloc(&sink, 16));

  // ---- 1. access granularity ----
  const size_t l2_bytes = 2u << 20;    // inside one XCD's 4 MB L2
  const size_t hbm_bytes = 2ull << 30; // far beyond the 256 MB Infinity Cache
  float* buf;
  UB_CHECK(hipMalloc(&buf, hbm_bytes));
  UB_CHECK(hipMemset(buf, 0, hbm_bytes));
  const int k = 256;
  const size_t strides[] = {4, 8, 16, 32, 64, 128, 256, 512};
  for (int level = 0; level < 2; ++level) {
    const size_t span = level == 0 ? l2_bytes : hbm_bytes;  // powers of two (address mask)
    double prev = 0, knee = 0;
    printf("%s footprint:\n", level == 0 ? "L2-resident" : "HBM");
    for (const size_t& st : strides) {
      double best = 1e30;
      for (int rep = 0; rep < 3; ++rep) {
        // HBM runs start each repetition on untouched lines (64 MB apart)
        const size_t base = level == 0 ? 0 : (size_t)(rep + 1 + 3 * (&st - strides)) * (64u << 20) / 4;
        hipLaunchKernelGGL(gran_kernel, dim3(1), dim3(64), 0, 0, buf, st / 4, k, span / 4 - 1, base, level == 0 ? 1 : 0,
                           d_out, sink);
        UB_CHECK(hipDeviceSynchronize());
        uint64_t c = 0;
        UB_CHECK(hipMemcpy(&c, d_out, 8, hipMemcpyDeviceToHost));
        best = std::min(best, (double)c / k);
      }
      printf("  stride %4zu B (wave footprint %6zu B): %7.1f clocks per wave-load\n", st, 64 * st, best);
      if (prev > 0 && !knee && best > 1.6 * prev) knee = (double)st / 2;
      prev = best;
    }
    if (knee) printf("# %s_access_granule_bytes %.0f\n", level == 0 ? "l2_to_l1" : "hbm", knee);
  }

  // ---- 2. memory-level parallelism (one lane, P chains, HBM) ----
  const size_t n_elems = hbm_bytes / 4;
  const uint32_t stride_elems = 4096 / 4;  // chains 4 KB apart, nodes 64 KB apart
  {
    std::vector<uint32_t> h(n_elems, 0);
    const size_t step = 65536 / 4;
    for (size_t i = 0; i + step < n_elems; i += step)
      for (size_t c = 0; c < 32; ++c) h[i + c * stride_elems] = (uint32_t)((i + step) % (n_elems - step) + c * stride_elems);
    UB_CHECK(hipMemcpy(buf, h.data(), n_elems * 4, hipMemcpyHostToDevice));
  }
  const int rounds = 2000;
  double one = 0;
  for (int p : {1, 2, 4, 8, 12, 16, 24, 32}) {
    hipLaunchKernelGGL(mlp_kernel, dim3(1), dim3(64), 0, 0, reinterpret_cast<const uint32_t*>(buf), p, rounds,
                       stride_elems, d_out);
    UB_CHECK(hipDeviceSynchronize());
    uint64_t c[2];
    UB_CHECK(hipMemcpy(c, d_out, 16, hipMemcpyDeviceToHost));
    const double per_round = (double)c[0] / rounds;
    if (p == 1) one = per_round;
    printf("  %2d independent HBM chains from one lane: %7.1f clocks per round (%.2f x one miss)\n", p, per_round,
           per_round / one);
    printf("# hbm_chains_%d_rel_round_time %.2f\n", p, per_round / one);
  }
  UB_CHECK(hipFree(buf));
  UB_CHECK(hipFree(d_out));
  UB_CHECK(hipFree(sink));
  return 0;
}
