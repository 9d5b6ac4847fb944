// HBM load latency and address-translation cost against footprint
// (reference GPU_Microbenchmark mem/mem_lat).  One lane pointer-chases 4096
// nodes in random order, cold (a 1 GB streaming read evicts L2 and MALL
// first):
//   packed - nodes 128 B apart (0.5 MB: a handful of pages)
//   spread - nodes footprint/4096 apart over 256 MB .. 8 GB (every node in
//            its own page once the spacing passes the page size)
// packed gives the HBM latency with warm translations; spread - packed is the
// translation-miss penalty at that footprint.
#include "ubench.h"

__global__ void scatter(uint32_t* buf, const uint64_t* at, const uint32_t* val, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) buf[at[i]] = val[i];
}

__global__ void __launch_bounds__(64) walk(const uint32_t* next, uint64_t stride_words, int iters, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t j = 0;
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) j = next[(uint64_t)j * stride_words];
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
  const int nodes = 4096;
  const size_t ev_bytes = size_t(1) << 30;
  float4* ev;
  float* sink;
  uint64_t* o;
  UB_CHECK(hipMalloc(&ev, ev_bytes));
  UB_CHECK(hipMemset(ev, 0, ev_bytes));
  UB_CHECK(hipMalloc(&sink, 4));
  UB_CHECK(hipMalloc(&o, 16));
  // node i holds the index of the next node (random cycle)
  std::vector<uint32_t> order(nodes);
  std::iota(order.begin(), order.end(), 0u);
  std::mt19937 g(3);
  std::shuffle(order.begin() + 1, order.end(), g);
  std::vector<uint32_t> nxt(nodes);
  for (int i = 0; i < nodes; ++i) nxt[order[i]] = order[(i + 1) % nodes];
  uint64_t* d_at;
  uint32_t* d_val;
  UB_CHECK(hipMalloc(&d_at, nodes * 8));
  UB_CHECK(hipMalloc(&d_val, nodes * 4));
  UB_CHECK(hipMemcpy(d_val, nxt.data(), nodes * 4, hipMemcpyHostToDevice));
  auto measure = [&](size_t footprint, uint64_t stride_bytes) {
    uint32_t* buf;
    UB_CHECK(hipMalloc(&buf, footprint));
    const uint64_t sw = stride_bytes / 4;
    std::vector<uint64_t> at(nodes);
    for (int i = 0; i < nodes; ++i) at[i] = (uint64_t)i * sw;
    UB_CHECK(hipMemcpy(d_at, at.data(), nodes * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(scatter, dim3((nodes + 255) / 256), dim3(256), 0, 0, buf, d_at, d_val, nodes);
    std::vector<double> v;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(evict, dim3(dev.cus() * 8), dim3(256), 0, 0, ev, ev_bytes / 16, sink);
      hipLaunchKernelGGL(walk, dim3(1), dim3(64), 0, 0, buf, sw, nodes, o);
      UB_CHECK(hipDeviceSynchronize());
      uint64_t r[2];
      UB_CHECK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
      v.push_back((double)r[0] / nodes);
    }
    UB_CHECK(hipFree(buf));
    std::sort(v.begin(), v.end());
    return v[1];
  };
  const double packed = measure(size_t(1) << 20, 128);
  printf("packed (128 B apart, 0.5 MB): %6.0f cycles/load\n", packed);
  const size_t mb[] = {256, 1024, 4096, 8192};
  double spread[4];
  for (int f = 0; f < 4; ++f) {
    const size_t fp = mb[f] << 20;
    spread[f] = measure(fp, fp / nodes);
    printf("spread over %5zu MB (%7zu KB apart): %6.0f cycles/load (+%.0f)\n", mb[f], fp / nodes / 1024, spread[f],
           spread[f] - packed);
  }
  printf("# hbm_cold_latency_cycles %.0f\n", packed);
  for (int f = 0; f < 4; ++f) printf("# translation_penalty_cycles_%zumb %.0f\n", mb[f], std::max(0.0, spread[f] - packed));
  UB_CHECK(hipFree(ev));
  UB_CHECK(hipFree(sink));
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(d_at));
  UB_CHECK(hipFree(d_val));
  return 0;
}
