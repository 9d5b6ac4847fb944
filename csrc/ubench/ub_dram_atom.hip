// Smallest unit HBM moves per access (reference GPU_Microbenchmark
// mem/mem_atom_size).  Every lane reads `useful` bytes at a random 256 B-
// aligned offset of a 4 GB buffer (far beyond L2 and the 256 MB MALL), so
// each access is a cold line: the achieved access rate is flat while the
// useful size is below the atom and then falls as bytes per access grow.
// Prints the access rate per size and the atom (the largest size whose rate
// is within 15 % of the 4-byte rate).
#include "ubench.h"

template <int W>
__global__ void __launch_bounds__(256) rand_read(const uint4* __restrict__ buf, size_t lines256, int iters,
                                                  uint32_t seed, uint32_t* sink) {
  uint32_t x = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    x = x * 1664525u + 1013904223u;
    const size_t line = (size_t)(x % (uint32_t)lines256);
    const uint4* p = buf + line * 16;  // 256 B = 16 x 16 B
#pragma unroll
    for (int k = 0; k < (W + 15) / 16; ++k) {
      const uint4 v = p[k];
      acc += v.x;
    }
  }
  if (acc == 0xdeadbeefu) sink[0] = acc;
}

template <int W>
static double run(int cus, const uint4* buf, size_t lines, uint32_t* sink) {
  const int blocks = cus * 8, iters = 64;
  hipLaunchKernelGGL((rand_read<W>), dim3(blocks), dim3(256), 0, 0, buf, lines, 4, 7u, sink);
  UB_CHECK(hipDeviceSynchronize());
  UbTimer t;
  t.start();
  hipLaunchKernelGGL((rand_read<W>), dim3(blocks), dim3(256), 0, 0, buf, lines, iters, 11u, sink);
  const double ms = t.stop_ms();
  const double acc = (double)blocks * 256 * iters;
  const double rate = acc / (ms * 1e-3) / 1e9;
  printf("useful %3d B per access: %8.3f G accesses/s  (%7.1f GB/s useful)\n", W, rate, rate * W);
  return rate;
}

int main() {
  UbDevice dev;
  printf("device %s, %d CUs\n", dev.p.gcnArchName, dev.cus());
  const size_t bytes = size_t(4) << 30, lines = bytes / 256;
  uint4* buf;
  uint32_t* sink;
  UB_CHECK(hipMalloc(&buf, bytes));
  UB_CHECK(hipMemset(buf, 1, bytes));
  UB_CHECK(hipMalloc(&sink, 4));
  const int sizes[] = {16, 32, 64, 128, 256};
  double r[5];
  r[0] = run<16>(dev.cus(), buf, lines, sink);
  r[1] = run<32>(dev.cus(), buf, lines, sink);
  r[2] = run<64>(dev.cus(), buf, lines, sink);
  r[3] = run<128>(dev.cus(), buf, lines, sink);
  r[4] = run<256>(dev.cus(), buf, lines, sink);
  int atom = sizes[0];
  for (int i = 1; i < 5; ++i)
    if (r[i] >= 0.85 * r[0]) atom = sizes[i];
  printf("# dram_random_access_rate_16B_gps %.3f\n# dram_access_atom_bytes %d\n", r[0], atom);
  UB_CHECK(hipFree(buf));
  UB_CHECK(hipFree(sink));
  return 0;
}
