// pathfinder-shaped dynamic programming (Rodinia pathfinder: minimum-cost
// path down a 2-D wall, one row per step, the previous row staged in shared
// memory with a one-column halo), plain HIP.
#include <algorithm>
#include <cmath>

#include "app_common.h"

constexpr int B = 256;

__global__ void dynproc_kernel(const int* wall_row, const int* src, int* dst, int cols) {
  __shared__ int prev[B + 2];
  const int x = blockIdx.x * B + threadIdx.x;
  prev[threadIdx.x + 1] = x < cols ? src[x] : 0x3fffffff;
  if (threadIdx.x == 0) prev[0] = x > 0 ? src[x - 1] : 0x3fffffff;
  if (threadIdx.x == B - 1) prev[B + 1] = x + 1 < cols ? src[x + 1] : 0x3fffffff;
  __syncthreads();
  if (x < cols) {
    const int l = prev[threadIdx.x], u = prev[threadIdx.x + 1], r = prev[threadIdx.x + 2];
    const int m = l < u ? (l < r ? l : r) : (u < r ? u : r);
    dst[x] = wall_row[x] + m;
  }
}

int main(int argc, char** argv) {
  const int cols = argc > 1 ? atoi(argv[1]) : 100000, rows = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> wall((size_t)rows * cols);
  uint32_t s = 12345;
  for (auto& v : wall) {
    s = s * 1664525u + 1013904223u;
    v = (int)((s >> 16) % 10);
  }
  int *dwall, *r0, *r1;
  APP_HIP(hipMalloc(&dwall, wall.size() * 4));
  APP_HIP(hipMalloc(&r0, cols * 4));
  APP_HIP(hipMalloc(&r1, cols * 4));
  APP_HIP(hipMemcpy(dwall, wall.data(), wall.size() * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(r0, wall.data(), cols * 4, hipMemcpyHostToDevice));
  const dim3 grid((cols + B - 1) / B), blk(B);
  for (int t = 1; t < rows; ++t)
    dynproc_kernel<<<grid, blk>>>(dwall + (size_t)t * cols, t % 2 ? r0 : r1, t % 2 ? r1 : r0, cols);
  APP_HIP(hipDeviceSynchronize());
  std::vector<int> out(cols);
  APP_HIP(hipMemcpy(out.data(), (rows - 1) % 2 ? r1 : r0, cols * 4, hipMemcpyDeviceToHost));
  // host check of the DP
  std::vector<int> a(wall.begin(), wall.begin() + cols), b(cols);
  for (int t = 1; t < rows; ++t) {
    for (int x = 0; x < cols; ++x) {
      int m = a[x];
      if (x > 0) m = std::min(m, a[x - 1]);
      if (x + 1 < cols) m = std::min(m, a[x + 1]);
      b[x] = wall[(size_t)t * cols + x] + m;
    }
    a.swap(b);
  }
  const bool ok = a == out;
  printf("pathfinder cols=%d rows=%d: %s\n", cols, rows, ok ? "PASSED" : "FAILED");
  APP_HIP(hipFree(dwall));
  APP_HIP(hipFree(r0));
  APP_HIP(hipFree(r1));
  return ok ? 0 : 1;
}
