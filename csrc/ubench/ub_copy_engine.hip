// Copies: bandwidth of hipMemcpy per direction and whether a device-to-device
// or host-to-device copy leaves its destination in the GPU's caches
// (reference GPU_Microbenchmark l2_cache/l2_copy_engine, which checks that a
// cudaMemcpy populates the L2; the simulator's -gpgpu_perf_sim_memcpy fills
// the L2 with every MemcpyHtoD of a trace).  After a 2 MB copy one lane
// pointer-chases the destination: at the L2-hit latency the copy filled the
// cache, at the cold (evicted) latency it did not.
#include <cstring>

#include "ubench.h"

__global__ void __launch_bounds__(64) walk(const uint32_t* next, int iters, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t j = 0;
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) j = next[j];
  const uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = j;
}

__global__ void evict(const float4* __restrict__ a, size_t n, float* sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += a[i].x;
  if (s == -1.f) sink[0] = s;
}

int main() {
  UbDevice dev;
  printf("device %s\n", dev.p.gcnArchName);
  // bandwidths
  const size_t big = size_t(512) << 20;
  void *d0, *d1, *h;
  UB_CHECK(hipMalloc(&d0, big));
  UB_CHECK(hipMalloc(&d1, big));
  UB_CHECK(hipHostMalloc(&h, big, hipHostMallocDefault));
  memset(h, 1, big);
  UbTimer t;
  auto bw = [&](void* dst, const void* src, hipMemcpyKind k) {
    UB_CHECK(hipMemcpy(dst, src, big, k));
    t.start();
    for (int r = 0; r < 4; ++r) UB_CHECK(hipMemcpyAsync(dst, src, big, k, 0));
    return 4.0 * big / (t.stop_ms() * 1e-3) / 1e9;
  };
  const double h2d = bw(d0, h, hipMemcpyHostToDevice), d2h = bw(h, d0, hipMemcpyDeviceToHost),
               d2d = bw(d1, d0, hipMemcpyDeviceToDevice);
  printf("hipMemcpy: H2D %.1f GB/s  D2H %.1f GB/s  D2D %.1f GB/s (read+write counted once)\n", h2d, d2h, d2d);
  // cache residency after a copy
  const size_t n = 16384, stride = 32, total = n * stride;  // 2 MB, one node per 128 B line
  auto chain = ub_chase(n, stride, total, 9);
  uint32_t *src, *dst;
  uint64_t* o;
  float* sink;
  float4* ev;
  const size_t ev_bytes = size_t(1) << 30;
  UB_CHECK(hipMalloc(&src, total * 4));
  UB_CHECK(hipMalloc(&dst, total * 4));
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 4));
  UB_CHECK(hipMalloc(&ev, ev_bytes));
  UB_CHECK(hipMemset(ev, 0, ev_bytes));
  UB_CHECK(hipMemcpy(src, chain.data(), total * 4, hipMemcpyHostToDevice));
  memcpy(h, chain.data(), total * 4);
  auto timed = [&](const uint32_t* p) {
    hipLaunchKernelGGL(walk, dim3(1), dim3(64), 0, 0, p, (int)n, o);
    UB_CHECK(hipDeviceSynchronize());
    uint64_t r[2];
    UB_CHECK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
    return (double)r[0] / n;
  };
  auto ev_run = [&] { hipLaunchKernelGGL(evict, dim3(dev.cus() * 8), dim3(256), 0, 0, ev, ev_bytes / 16, sink); };
  std::vector<double> cold, warm, after_d2d, after_h2d;
  for (int rep = 0; rep < 5; ++rep) {
    ev_run();
    cold.push_back(timed(src));
    warm.push_back(timed(src));  // second walk of the same chain: cache resident
    ev_run();
    UB_CHECK(hipMemcpy(dst, src, total * 4, hipMemcpyDeviceToDevice));
    after_d2d.push_back(timed(dst));
    ev_run();
    UB_CHECK(hipMemcpy(dst, h, total * 4, hipMemcpyHostToDevice));
    after_h2d.push_back(timed(dst));
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const double c = med(cold), w = med(warm), a = med(after_d2d), b = med(after_h2d);
  printf("walk of a 2 MB chain: cold %.0f, resident %.0f, after D2D copy %.0f, after H2D copy %.0f cycles/load\n", c, w,
         a, b);
  const bool d2d_fills = a < w + 0.3 * (c - w), h2d_fills = b < w + 0.3 * (c - w);
  printf("# copy_h2d_gbps %.1f\n# copy_d2h_gbps %.1f\n# copy_d2d_gbps %.1f\n", h2d, d2h, d2d);
  printf("# d2d_copy_fills_cache %d\n# h2d_copy_fills_cache %d\n", d2d_fills ? 1 : 0, h2d_fills ? 1 : 0);
  printf("# suggest_gpgpu_perf_sim_memcpy %d\n", h2d_fills ? 1 : 0);
  UB_CHECK(hipFree(d0));
  UB_CHECK(hipFree(d1));
  UB_CHECK(hipHostFree(h));
  UB_CHECK(hipFree(src));
  UB_CHECK(hipFree(dst));
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
  UB_CHECK(hipFree(ev));
  return 0;
}
