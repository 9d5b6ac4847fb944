// Address translation on the load path (no reference counterpart: GPGPU-Sim
// has no TLB; the MI355X has a per-CU UTCL1, an L2 TLB and page walks).
//
// One lane pointer-chases N nodes, one per `stride` bytes (each node on its
// own 128 B line, the lines spread over the cache sets), so the same number
// of distinct lines is touched whatever the stride and only the number of
// pages (translations) changes:
//   same   - the wave walks the chain once, then times a second walk: the
//            lines are L2 hits, the translations are warm if the TLBs reach
//   next   - a 256-workgroup kernel walks the chain on every CU first, then
//            a one-workgroup kernel times a walk: warm translations survive
//            the kernel boundary or not (read lines stay in the L2,
//            ub_l2_release)
//   cold   - a 1 GB streaming read evicted L2, MALL and translations first
// The 128 B stride (every node in one 2 MB region) is the no-translation
// baseline; stride 4 KB / 64 KB / 2 MB / 8 MB spread the same node count over
// ever more pages.  Prints "# tlb_*" lines for the tuner.
#include "ubench.h"

__global__ void __launch_bounds__(64) tlb_walk(const uint32_t* __restrict__ next, uint32_t start, int n, int warm,
                                              uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t j = start;
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

// next[pos[i]] = pos[i + 1]: the chain built on the device (a 8 GB-span chain
// is never materialised on the host)
__global__ void tlb_link(uint32_t* next, const uint32_t* pos, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) next[pos[i]] = pos[(i + 1) % n];
}

__global__ void tlb_evict(const float4* __restrict__ a, size_t n, float* sink) {
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
  const size_t span = size_t(8) << 30;  // 8 GB of address space for the widest chain
  uint32_t* d_next = nullptr;
  if (hipMalloc(&d_next, span) != hipSuccess) {
    printf("cannot allocate the chain buffer\n");
    return 1;
  }
  uint32_t* d_pos;
  uint64_t* d_out;
  float* d_sink;
  float4* d_ev;
  const size_t ev_bytes = size_t(1) << 30;
  const int max_n = 2048;
  UB_CHECK(hipMalloc(&d_pos, max_n * 4));
  UB_CHECK(hipMalloc(&d_out, 16));
  UB_CHECK(hipMalloc(&d_sink, 4));
  UB_CHECK(hipMalloc(&d_ev, ev_bytes));
  UB_CHECK(hipMemset(d_ev, 0, ev_bytes));
  auto evict = [&] {
    hipLaunchKernelGGL(tlb_evict, dim3(dev.cus() * 8), dim3(256), 0, 0, d_ev, ev_bytes / 16, d_sink);
  };
  auto median = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const size_t strides[] = {128, 4096, 65536, size_t(2) << 20, size_t(8) << 20};
  const int counts[] = {64, 512, 2048};
  double base_same[3] = {0, 0, 0}, base_next[3] = {0, 0, 0}, base_cold[3] = {0, 0, 0};
  printf("%-10s %6s %10s %10s %10s   (cycles per load)\n", "stride", "nodes", "same", "next", "cold");
  for (size_t stride : strides) {
    for (int ci = 0; ci < 3; ++ci) {
      const int n = counts[ci];
      if ((size_t)n * stride > span) continue;
      // node i: page i, a line inside it that spreads the sets
      const size_t lines_per = std::max<size_t>(1, std::min<size_t>(64, stride / 128));
      std::vector<uint32_t> pos(n);
      std::vector<uint32_t> order(n);
      std::iota(order.begin(), order.end(), 0u);
      std::mt19937 g(7 + n);
      std::shuffle(order.begin() + 1, order.end(), g);
      for (int i = 0; i < n; ++i) {
        const size_t k = order[i];
        const size_t byte = k * stride + ((k * 37) % lines_per) * 128;
        pos[i] = (uint32_t)(byte / 4);
      }
      UB_CHECK(hipMemcpy(d_pos, pos.data(), n * 4, hipMemcpyHostToDevice));
      hipLaunchKernelGGL(tlb_link, dim3((n + 255) / 256), dim3(256), 0, 0, d_next, d_pos, n);
      UB_CHECK(hipDeviceSynchronize());
      const uint32_t start = pos[0];
      auto timed = [&](int warm) {
        hipLaunchKernelGGL(tlb_walk, dim3(1), dim3(64), 0, 0, d_next, start, n, warm, d_out);
        UB_CHECK(hipDeviceSynchronize());
        uint64_t r[2];
        UB_CHECK(hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost));
        return (double)r[0] / n;
      };
      std::vector<double> same, nxt, cold;
      for (int rep = 0; rep < 5; ++rep) {
        evict();
        same.push_back(timed(n));
        evict();
        hipLaunchKernelGGL(tlb_walk, dim3(dev.cus()), dim3(64), 0, 0, d_next, start, n, 0, nullptr);
        nxt.push_back(timed(0));
        evict();
        cold.push_back(timed(0));
      }
      const double s = median(same), x = median(nxt), c = median(cold);
      printf("%-10zu %6d %10.1f %10.1f %10.1f\n", stride, n, s, x, c);
      printf("# tlb_s%zu_n%d %.1f %.1f %.1f\n", stride, n, s, x, c);
      if (stride == 128) {
        base_same[ci] = s;
        base_next[ci] = x;
        base_cold[ci] = c;
      }
    }
  }
  printf("# tlb_base_same_n512 %.1f\n# tlb_base_next_n512 %.1f\n# tlb_base_cold_n512 %.1f\n", base_same[1],
         base_next[1], base_cold[1]);
  UB_CHECK(hipFree(d_next));
  UB_CHECK(hipFree(d_pos));
  UB_CHECK(hipFree(d_out));
  UB_CHECK(hipFree(d_sink));
  UB_CHECK(hipFree(d_ev));
  return 0;
}
