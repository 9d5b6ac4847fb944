// Copy-engine and DRAM access-atom measurements (reference GPU_Microbenchmark
// l2_cache/l2_copy_engine and mem/mem_atom_size): hipMemcpy bandwidth host to
// device, device to host (pinned host memory) and device to device, and the
// HBM bandwidth of a streaming read whose lanes touch only the first `w`
// bytes of every 128-byte line -- the smallest width at which bandwidth in
// useful bytes stops falling is the DRAM access atom.
#include <cstring>

#include "ubench.h"

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void ub_atom_kernel(const v4u* __restrict__ src, size_t lines, int words, uint32_t* sink) {
  // one lane per line, reading `words` 16-byte words of it
  uint32_t acc = 0;
  for (size_t l = blockIdx.x * (size_t)blockDim.x + threadIdx.x; l < lines; l += (size_t)gridDim.x * blockDim.x) {
    const v4u* p = src + l * 8;
    for (int w = 0; w < words; ++w) {
      const v4u v = __builtin_nontemporal_load(p + w);
      acc += v.x ^ v.w;
    }
  }
  if (acc == 0xdeadbeef) sink[0] = acc;
}

int main() {
  UbDevice d;
  const size_t bytes = (size_t)256 << 20;
  void *dev_a, *dev_b, *host;
  UB_CHECK(hipMalloc(&dev_a, bytes));
  UB_CHECK(hipMalloc(&dev_b, bytes));
  UB_CHECK(hipHostMalloc(&host, bytes));
  memset(host, 1, bytes);
  UbTimer t;
  auto bw = [&](void* dst, const void* src, hipMemcpyKind k) {
    UB_CHECK(hipMemcpy(dst, src, bytes, k));
    t.start();
    for (int r = 0; r < 5; ++r) UB_CHECK(hipMemcpyAsync(dst, src, bytes, k, 0));
    return 5.0 * (double)bytes / (t.stop_ms() * 1e-3) / 1e9;
  };
  const double h2d = bw(dev_a, host, hipMemcpyHostToDevice);
  const double d2h = bw(host, dev_a, hipMemcpyDeviceToHost);
  const double d2d = bw(dev_b, dev_a, hipMemcpyDeviceToDevice);
  printf("hipMemcpy 256 MB: H2D %.1f GB/s, D2H %.1f GB/s, D2D %.1f GB/s (read+write %.1f GB/s)\n", h2d, d2h, d2d,
         2 * d2d);
  printf("# copy_h2d_gbps %.1f\n# copy_d2h_gbps %.1f\n# copy_d2d_gbps %.1f\n", h2d, d2h, d2d);
  uint32_t* sink;
  UB_CHECK(hipMalloc(&sink, 4));
  const size_t lines = bytes / 128;
  double prev_useful = 0;
  int atom = 128;
  for (int words : {1, 2, 4, 8}) {
    hipLaunchKernelGGL(ub_atom_kernel, dim3(d.cus() * 8), dim3(256), 0, 0, (const v4u*)dev_a, lines, words, sink);
    UB_CHECK(hipDeviceSynchronize());
    t.start();
    for (int r = 0; r < 5; ++r)
      hipLaunchKernelGGL(ub_atom_kernel, dim3(d.cus() * 8), dim3(256), 0, 0, (const v4u*)dev_a, lines, words, sink);
    const double s = t.stop_ms() * 1e-3 / 5.0;
    const double useful = (double)lines * words * 16 / s / 1e9, lines_per_s = (double)lines / s / 1e9;
    printf("read %3d B of every 128 B line: %7.1f GB/s useful, %6.2f G lines/s\n", words * 16, useful, lines_per_s);
    if (prev_useful > 0 && useful < 1.15 * prev_useful && atom == 128) atom = words * 16 / 2;
    prev_useful = useful;
  }
  printf("# dram_access_atom_bytes %d\n", atom);
  UB_CHECK(hipFree(dev_a));
  UB_CHECK(hipFree(dev_b));
  UB_CHECK(hipHostFree(host));
  UB_CHECK(hipFree(sink));
  return 0;
}
