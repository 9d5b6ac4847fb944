// nn-shaped nearest-neighbour distance kernel (Rodinia nn: Euclidean distance
// of every (lat, lng) record to a query point), plain HIP.
#include <cmath>

#include "app_common.h"

__global__ void euclid(const float2* loc, float* dist, int n, float lat, float lng) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const float2 p = loc[i];
    const float dx = lat - p.x, dy = lng - p.y;
    dist[i] = sqrtf(dx * dx + dy * dy);
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 42764 * 8;
  std::vector<float2> h(n);
  for (int i = 0; i < n; ++i) h[i] = make_float2(30.f + 10.f * std::sin(0.37f * i), 90.f * std::cos(0.11f * i));
  float2* d;
  float* dist;
  APP_HIP(hipMalloc(&d, n * sizeof(float2)));
  APP_HIP(hipMalloc(&dist, n * 4));
  APP_HIP(hipMemcpy(d, h.data(), n * sizeof(float2), hipMemcpyHostToDevice));
  const int blk = 256;
  euclid<<<(n + blk - 1) / blk, blk>>>(d, dist, n, 30.f, 90.f);
  APP_HIP(hipGetLastError());
  APP_HIP(hipDeviceSynchronize());
  std::vector<float> out(n);
  APP_HIP(hipMemcpy(out.data(), dist, n * 4, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < n && ok; i += 997) {
    const float dx = 30.f - h[i].x, dy = 90.f - h[i].y;
    ok = std::fabs(out[i] - std::sqrt(dx * dx + dy * dy)) < 1e-3f;
  }
  printf("nn n=%d: %s\n", n, ok ? "PASSED" : "FAILED");
  APP_HIP(hipFree(d));
  APP_HIP(hipFree(dist));
  return ok ? 0 : 1;
}
