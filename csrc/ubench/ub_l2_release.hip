// Does an XCD's L2 keep its lines across a kernel boundary?  (no reference
// counterpart: NVIDIA's L2 is one coherent cache; it sets
// -sim_l2_kernel_release).  One lane pointer-chases a 256 KB chain (inside one
// XCD's 4 MB L2, far beyond the 32 KB vector L1):
//   same kernel  - the wave walks the chain once to warm it, then times a walk
//                  (L2 hits: the reference latency of a kept line)
//   next kernel, read  - kernel A (eight workgroups: one per XCD) walks the
//                  chain, kernel B (one workgroup) times a walk
//   next kernel, write - kernel A (eight workgroups) rewrites the chain (same
//                  values), kernel B times a walk
//   cold         - a 1 GB streaming read evicted L2 and MALL first
// A next-kernel walk at the same-kernel latency means the L2 kept the lines;
// one at the MALL latency means the kernel boundary wrote back and
// invalidated them (the multi-XCD release / acquire).
// Measured on MI355X: read lines kept, written lines dropped in this minimal
// two-kernel case; the Rodinia suite's L2 -> fabric read traffic
// (TCC_EA0_RDREQ) matches invalidating every line within 1.7 % and keeping
// clean lines undercounts it by up to 67 % (profiles/correlation), so the
// simulator invalidates all lines; the option line follows the written-line
// result.
#include "ubench.h"

__global__ void __launch_bounds__(64) rel_walk(const uint32_t* __restrict__ next, int n, int warm, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t j = 0;
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  for (int i = 0; i < warm; ++i) j = next[j];
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < n; ++i) j = next[j];
  const uint64_t t1 = ub_clock();
  if (out) {
    out[0] = t1 - t0;
    out[1] = j;
  }
}

__global__ void __launch_bounds__(64) rel_rewrite(uint32_t* next, const uint32_t* __restrict__ src, int n,
                                                  uint32_t stride) {
  for (int i = threadIdx.x; i < n; i += 64) next[(size_t)i * stride] = src[i];
}

__global__ void rel_evict(const float4* __restrict__ a, size_t n, float* sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.w;
  }
  if (s == -1.f) sink[0] = s;
}

int main() {
  UbDevice dev;
  printf("device %s, %d CUs\n", dev.p.gcnArchName, dev.cus());
  const uint32_t stride = 32;  // 128 B: one line per node
  const int n = 2048;          // 256 KB
  const size_t total = (size_t)n * stride;
  auto chain = ub_chase(n, stride, total, 11);
  std::vector<uint32_t> src(n);
  for (int i = 0; i < n; ++i) src[i] = chain[(size_t)i * stride];
  uint32_t *d_next, *d_src;
  uint64_t* d_out;
  float* d_sink;
  float4* d_ev;
  const size_t ev_bytes = size_t(1) << 30;
  UB_CHECK(hipMalloc(&d_next, total * 4));
  UB_CHECK(hipMalloc(&d_src, n * 4));
  UB_CHECK(hipMalloc(&d_out, 16));
  UB_CHECK(hipMalloc(&d_sink, 4));
  UB_CHECK(hipMalloc(&d_ev, ev_bytes));
  UB_CHECK(hipMemset(d_ev, 0, ev_bytes));
  UB_CHECK(hipMemcpy(d_next, chain.data(), total * 4, hipMemcpyHostToDevice));
  UB_CHECK(hipMemcpy(d_src, src.data(), n * 4, hipMemcpyHostToDevice));
  auto evict = [&] {
    hipLaunchKernelGGL(rel_evict, dim3(dev.cus() * 8), dim3(256), 0, 0, d_ev, ev_bytes / 16, d_sink);
  };
  auto timed = [&](int warm) {
    hipLaunchKernelGGL(rel_walk, dim3(1), dim3(64), 0, 0, d_next, n, warm, d_out);
    UB_CHECK(hipDeviceSynchronize());
    uint64_t r[2];
    UB_CHECK(hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost));
    return (double)r[0] / n;
  };
  auto median = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::vector<double> same, nk_read, nk_write, cold;
  for (int rep = 0; rep < 7; ++rep) {
    evict();
    same.push_back(timed(n));
    evict();
    // kernel A on all eight XCDs (workgroups round-robin over them), so
    // kernel B's workgroup finds the lines in its own XCD's L2 if kept
    hipLaunchKernelGGL(rel_walk, dim3(8), dim3(64), 0, 0, d_next, n, 0, nullptr);
    nk_read.push_back(timed(0));
    evict();
    hipLaunchKernelGGL(rel_rewrite, dim3(8), dim3(64), 0, 0, d_next, d_src, n, stride);
    nk_write.push_back(timed(0));
    evict();
    cold.push_back(timed(0));
  }
  const double s = median(same), r = median(nk_read), w = median(nk_write), c = median(cold);
  printf("same kernel (L2 hit)   %7.1f cycles/load\n", s);
  printf("next kernel after read %7.1f cycles/load\n", r);
  printf("next kernel after write%7.1f cycles/load\n", w);
  printf("cold (evicted)         %7.1f cycles/load\n", c);
  // kept when the next kernel's walk is within a quarter of the gap of the
  // same-kernel hit latency
  const bool kept_read = r < s + 0.25 * (c - s);
  const bool kept_write = w < s + 0.25 * (c - s);
  printf("L2 across a kernel boundary: read lines %s, written lines %s\n", kept_read ? "kept" : "dropped",
         kept_write ? "kept" : "dropped");
  printf("# l2_same_kernel_latency %.1f\n# l2_next_kernel_read_latency %.1f\n# l2_next_kernel_write_latency %.1f\n",
         s, r, w);
  printf("# l2_cold_latency %.1f\n# l2_kept_across_kernels %d\n", c, (kept_read && kept_write) ? 1 : 0);
  ub_opt("-sim_l2_kernel_release", kept_write ? 0 : 1);
  UB_CHECK(hipFree(d_next));
  UB_CHECK(hipFree(d_src));
  UB_CHECK(hipFree(d_out));
  UB_CHECK(hipFree(d_sink));
  UB_CHECK(hipFree(d_ev));
  return 0;
}
