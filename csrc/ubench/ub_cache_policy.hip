// Cache write policies and vector-L1 bandwidth of the gfx950 it runs on
// (reference GPU_Microbenchmark l1_cache/write_policy_mb, l2_cache/
// write_policy_mb, l1_cache/l1_bw and l2_cache/l2_bw).
//
// 1. Write policy.  One wavefront, one kernel launch (the vector L1 is
//    invalidated at every dispatch and each XCD has its own L2, so writing
//    and probing must happen inside the same wave).  The wave lays a
//    pointer chain into `dst` and lane 0 then walks it once; the cycles per
//    load tell which level holds the freshly written lines:
//      cold     - no store, no warm read (after evicting L2 and MALL): miss path
//      warm     - wave reads the chain first, then walks it: read-allocate path
//      store    - wave stores the chain (copied from `src`), then walks it
//      rd+store - wave reads the chain, overwrites it with the same values,
//                 then walks it (does a store keep, update or drop the line?)
//      line-st  - wave stores every node's whole 128 B line, then walks it.
//                 A 4-byte store that leaves the line missing while a
//                 whole-line store makes it hit is a lazy-fetch-on-read
//                 allocation (gpgpusim write-allocate 'L'): the line is
//                 allocated with a byte mask and a read of a partly valid line
//                 goes to memory.
//    A chain of 8 KB (fits the 32 KB vector L1) probes the L1 policy; one of
//    512 KB (fits the 4 MB XCD L2, misses the L1) probes the L2 policy.
//    Before every launch a 1 GB streaming read evicts L2 and the 256 MB MALL.
// 2. Vector-L1 bandwidth: every CU re-reads 4 KB slices (four per CU) with 16-byte
//    loads; bytes / (elapsed shader clocks x CUs) is the per-CU L1 bandwidth.
#include "ubench.h"

__global__ void __launch_bounds__(64) wpol_kernel(const uint32_t* __restrict__ src, uint32_t* dst, int n_nodes,
                                                   uint32_t stride_e, int mode, uint64_t* out) {
  const int l = threadIdx.x;
  uint32_t acc = 0;
  if (mode == 1 || mode == 3)  // warm read of every node
    for (int i = l; i < n_nodes; i += 64) acc += dst[(size_t)i * stride_e];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (mode == 2 || mode == 3)  // store the chain (same values the host put there)
    for (int i = l; i < n_nodes; i += 64) dst[(size_t)i * stride_e] = src[i];
  if (mode == 4)  // store whole 128 B lines: the node word plus the 31 zero words around it
    for (int i = 0; i < n_nodes; ++i)
      if (l < (int)stride_e) dst[(size_t)i * stride_e + l] = l ? 0u : src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (l != 0) return;
  uint32_t j = 0;
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < n_nodes; ++i) j = dst[j];
  const uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = j + acc;
}

__global__ void evict_kernel(const float4* __restrict__ a, size_t n, float* sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == -1.f) sink[0] = s;
}

__global__ void __launch_bounds__(256) l1bw_kernel(const float4* __restrict__ a, int reps, float* sink) {
  // each block owns a 4 KB slice (256 float4): four blocks per CU stay well
  // inside the 32 KB vector L1
  const float4* s = a + (size_t)blockIdx.x * 256;
  float acc = 0.f;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = s[(threadIdx.x + k * 16 + r * 64) & 255];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == -1.f) sink[0] = acc;
}

static const char* kModes[5] = {"cold", "warm", "store", "rd+store", "line-st"};

int main() {
  UbDevice dev;
  const double mhz = ub_shader_mhz();
  printf("device %s, %d CUs, shader clock %.0f MHz\n", dev.p.gcnArchName, dev.cus(), mhz);
  uint64_t* d_out;
  float* d_sink;
  UB_CHECK(hipMalloc(&d_out, 16));
  UB_CHECK(hipMalloc(&d_sink, 4));
  const size_t evict_bytes = size_t(1) << 30;
  float4* d_evict;
  UB_CHECK(hipMalloc(&d_evict, evict_bytes));
  UB_CHECK(hipMemset(d_evict, 0, evict_bytes));

  const uint32_t stride_e = 32;  // 128 B between chain nodes: one line each
  double lat[2][5] = {};
  const int nodes_of[2] = {64, 4096};  // 8 KB (L1 probe), 512 KB (L2 probe)
  for (int t = 0; t < 2; ++t) {
    const int n = nodes_of[t];
    const size_t total = (size_t)n * stride_e;
    auto chain = ub_chase(n, stride_e, total, 7 + t);
    std::vector<uint32_t> src(n);
    for (int i = 0; i < n; ++i) src[i] = chain[(size_t)i * stride_e];
    uint32_t *d_dst, *d_src;
    UB_CHECK(hipMalloc(&d_dst, total * 4));
    UB_CHECK(hipMalloc(&d_src, n * 4));
    UB_CHECK(hipMemcpy(d_dst, chain.data(), total * 4, hipMemcpyHostToDevice));
    UB_CHECK(hipMemcpy(d_src, src.data(), n * 4, hipMemcpyHostToDevice));
    for (int mode = 0; mode < 5; ++mode) {
      std::vector<double> v;
      for (int rep = 0; rep < 7; ++rep) {
        hipLaunchKernelGGL(evict_kernel, dim3(dev.cus() * 8), dim3(256), 0, 0, d_evict, evict_bytes / 16, d_sink);
        hipLaunchKernelGGL(wpol_kernel, dim3(1), dim3(64), 0, 0, d_src, d_dst, n, stride_e, mode, d_out);
        UB_CHECK(hipDeviceSynchronize());
        uint64_t r[2];
        UB_CHECK(hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost));
        v.push_back((double)r[0] / n);
      }
      std::sort(v.begin(), v.end());
      lat[t][mode] = v[v.size() / 2];
      printf("%-9s chain %6zu KB: %-8s %7.1f cycles/load\n", t ? "L2 probe" : "L1 probe", total * 4 / 1024,
             kModes[mode], lat[t][mode]);
    }
    UB_CHECK(hipFree(d_dst));
    UB_CHECK(hipFree(d_src));
  }
  // a level "holds" the written lines when the walk costs about what a walk
  // over read-allocated lines costs there (within a quarter of the gap to the
  // next level down)
  auto near = [](double x, double hit, double miss) { return x < hit + 0.25 * (miss - hit); };
  const int l1_wa = near(lat[0][4], lat[0][1], lat[1][1]);
  const int l1_partial_wa = near(lat[0][2], lat[0][1], lat[1][1]);
  const int l1_keep = near(lat[0][3], lat[0][1], lat[1][1]);
  const int l2_wa = near(lat[1][4], lat[1][1], lat[1][0]);
  const int l2_partial_hit = near(lat[1][2], lat[1][1], lat[1][0]);
  const int l2_lazy = l2_wa && !l2_partial_hit;
  const int l2_hit_keep = near(lat[1][3], lat[1][1], lat[1][0]);
  printf("L1: whole-line store %s the line, 4-byte store %s; a store to a cached line %s it\n",
         l1_wa ? "allocates" : "does not allocate", l1_partial_wa ? "allocates" : "does not allocate",
         l1_keep ? "keeps" : "evicts / bypasses");
  if (l2_lazy)
    printf("L2: whole-line store allocates; a partly written line is fetched from memory on read (lazy fetch on read)\n");
  else
    printf("L2: store miss %s the line; a store hit %s the line\n", l2_wa ? "allocates" : "does not allocate",
           l2_hit_keep ? "keeps" : "drops");
  printf("# l1_write_allocate %d\n# l1_partial_write_allocate %d\n# l1_store_keeps_line %d\n", l1_wa, l1_partial_wa,
         l1_keep);
  printf("# l2_write_allocate %d\n# l2_lazy_fetch_on_read %d\n# l2_store_hit_keeps_line %d\n", l2_wa, l2_lazy,
         l2_hit_keep);
  printf("# l1_line_store_then_load_latency %.1f\n# l2_line_store_then_load_latency %.1f\n", lat[0][4], lat[1][4]);
  printf("# l2_partial_store_then_load_latency %.1f\n", lat[1][2]);

  // vector-L1 bandwidth
  const int blocks = dev.cus() * 4;
  float4* d_l1;
  UB_CHECK(hipMalloc(&d_l1, (size_t)blocks * 4096));
  UB_CHECK(hipMemset(d_l1, 0, (size_t)blocks * 4096));
  const int reps = 4096;
  hipLaunchKernelGGL(l1bw_kernel, dim3(blocks), dim3(256), 0, 0, d_l1, 64, d_sink);
  UB_CHECK(hipDeviceSynchronize());
  UbTimer tm;
  double best_ms = 1e30;
  for (int rep = 0; rep < 5; ++rep) {
    tm.start();
    hipLaunchKernelGGL(l1bw_kernel, dim3(blocks), dim3(256), 0, 0, d_l1, reps, d_sink);
    best_ms = std::min(best_ms, (double)tm.stop_ms());
  }
  const double bytes = (double)blocks * reps * 4 * 256 * 16;
  const double gbps = bytes / (best_ms * 1e-3) / 1e9;
  const double per_cu_clk = bytes / (best_ms * 1e-3 * mhz * 1e6) / dev.cus();
  printf("vector L1 re-read: %.0f GB/s device, %.1f B/clk/CU (%d blocks x 4 KB slices)\n", gbps, per_cu_clk, blocks);
  printf("# l1_read_gbps %.1f\n# l1_bytes_per_clk_per_cu %.1f\n", gbps, per_cu_clk);

  UB_CHECK(hipFree(d_l1));
  UB_CHECK(hipFree(d_evict));
  UB_CHECK(hipFree(d_out));
  UB_CHECK(hipFree(d_sink));
  return 0;
}
