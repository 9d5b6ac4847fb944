// HBM3E and L2 bandwidth (reference GPU_Microbenchmark mem/mem_bw and
// l2_cache/l2_bw): grid-stride 16-byte loads / stores over the whole chip,
// 4096 workgroups of 256 threads (>> 256 CUs), timed with events over
// back-to-back launches.
#include "ubench.h"

__global__ void rd_kernel(const float4* __restrict__ a, size_t n, float* sink) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.678f) sink[0] = acc.x;
}

// each workgroup re-reads the same `n`-element window `reps` times (L2 resident)
__global__ void rd_loop_kernel(const float4* __restrict__ a, size_t n, int reps, float* sink) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (int r = 0; r < reps; ++r)
    for (size_t i = threadIdx.x + (size_t)(blockIdx.x % 8) * blockDim.x; i < n; i += (size_t)8 * blockDim.x) {
      float4 v = a[i];
      acc.x += v.x;
      acc.w += v.w;
    }
  if (acc.x + acc.w == 12345.678f) sink[0] = acc.x;
}

__global__ void wr_kernel(float4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4(1, 2, 3, 4);
}

__global__ void cp_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

int main() {
  UbDevice d;
  const size_t big = (size_t)2 << 30;  // 2 GB per buffer: far beyond L2 + MALL
  float4 *a, *b;
  float* sink;
  UB_CHECK(hipMalloc(&a, big));
  UB_CHECK(hipMalloc(&b, big));
  UB_CHECK(hipMalloc(&sink, 4));
  UB_CHECK(hipMemset(a, 0, big));
  UB_CHECK(hipMemset(b, 0, big));
  const size_t n = big / sizeof(float4);
  const dim3 grid(4096), blk(256);
  UbTimer t;
  const int reps = 10;
  auto bw = [&](auto launch, double bytes_per_rep) {
    launch();
    UB_CHECK(hipDeviceSynchronize());
    t.start();
    for (int r = 0; r < reps; ++r) launch();
    const float ms = t.stop_ms();
    return bytes_per_rep * reps / (ms * 1e-3) / 1e9;
  };
  const double rd = bw([&] { hipLaunchKernelGGL(rd_kernel, grid, blk, 0, 0, a, n, sink); }, (double)big);
  const double wr = bw([&] { hipLaunchKernelGGL(wr_kernel, grid, blk, 0, 0, a, n); }, (double)big);
  const double cp = bw([&] { hipLaunchKernelGGL(cp_kernel, grid, blk, 0, 0, a, b, n); }, 2.0 * big);
  printf("HBM read %.1f GB/s, write %.1f GB/s, copy %.1f GB/s\n", rd, wr, cp);
  // L2: every workgroup re-reads an eighth of the same 1 MB (fits each
  // XCD's 4 MB L2) 64 times inside one launch
  const size_t l2n = ((size_t)1 << 20) / sizeof(float4);
  const int l2reps = 64;
  const double l2 = bw([&] { hipLaunchKernelGGL(rd_loop_kernel, grid, blk, 0, 0, a, l2n, l2reps, sink); },
                       (double)grid.x * l2reps * (double)(l2n / 8) * sizeof(float4));
  printf("L2-resident read %.1f GB/s\n", l2);
  printf("# hbm_read_gbps %.1f\n# hbm_write_gbps %.1f\n# hbm_copy_gbps %.1f\n# l2_read_gbps %.1f\n", rd, wr, cp, l2);
  // bytes per DRAM clock per channel (DDR) such that the simulated channels,
  // running at the ~80 % bus efficiency a streaming read reaches, deliver the
  // measured read bandwidth; rounded up to a power of two
  const int channels = std::max(1, d.p.memoryBusWidth / 64);
  const double mem_mhz = d.p.memoryClockRate / 1000.0;
  const double need = rd * 1e9 / (0.8 * channels * 2.0 * mem_mhz * 1e6);
  int width = 1;
  while (width < need) width *= 2;
  ub_opt("-gpgpu_dram_buswidth", width);
  UB_CHECK(hipFree(a));
  UB_CHECK(hipFree(b));
  UB_CHECK(hipFree(sink));
  return 0;
}
