// hotspot-shaped thermal stencil (Rodinia hotspot: 2-D grid of temperatures
// + power map, 5-point update per step, 16x16 tiles staged through shared
// memory), plain HIP.  One launch per simulated step, ping-ponging between two
// temperature buffers.
#include <cmath>

#include "app_common.h"

constexpr int T = 16;

__global__ void calculate_temp(const float* power, const float* tin, float* tout, int nx, int ny, float cap, float rx,
                               float ry, float rz, float amb) {
  __shared__ float tile[T + 2][T + 2];
  const int gx = blockIdx.x * T + threadIdx.x, gy = blockIdx.y * T + threadIdx.y;
  const int tx = threadIdx.x + 1, ty = threadIdx.y + 1;
  const bool in = gx < nx && gy < ny;
  const int idx = gy * nx + gx;
  const float c = in ? tin[idx] : 0.f;
  tile[ty][tx] = c;
  // halo: edge threads fetch the neighbour tile's border (clamped at the grid edge)
  if (threadIdx.x == 0) tile[ty][0] = gy < ny ? tin[gy * nx + (gx > 0 ? gx - 1 : gx)] : 0.f;
  if (threadIdx.x == T - 1) tile[ty][T + 1] = gy < ny ? tin[gy * nx + (gx + 1 < nx ? gx + 1 : gx)] : 0.f;
  if (threadIdx.y == 0) tile[0][tx] = gx < nx ? tin[(gy > 0 ? gy - 1 : gy) * nx + gx] : 0.f;
  if (threadIdx.y == T - 1) tile[T + 1][tx] = gx < nx ? tin[(gy + 1 < ny ? gy + 1 : gy) * nx + gx] : 0.f;
  __syncthreads();
  if (in) {
    const float p = power[idx];
    const float n_ = tile[ty - 1][tx], s_ = tile[ty + 1][tx], e_ = tile[ty][tx + 1], w_ = tile[ty][tx - 1];
    const float d = cap * (p + (s_ + n_ - 2.f * c) * ry + (e_ + w_ - 2.f * c) * rx + (amb - c) * rz);
    tout[idx] = c + d;
  }
}

int main(int argc, char** argv) {
  const int nx = argc > 1 ? atoi(argv[1]) : 512, ny = nx, steps = argc > 2 ? atoi(argv[2]) : 4;
  const size_t n = (size_t)nx * ny;
  std::vector<float> hp(n), ht(n);
  for (size_t i = 0; i < n; ++i) {
    hp[i] = 0.5f + 0.5f * std::sin(0.01f * (float)i);
    ht[i] = 320.f + std::cos(0.003f * (float)i);
  }
  float *p, *t0, *t1;
  APP_HIP(hipMalloc(&p, n * 4));
  APP_HIP(hipMalloc(&t0, n * 4));
  APP_HIP(hipMalloc(&t1, n * 4));
  APP_HIP(hipMemcpy(p, hp.data(), n * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(t0, ht.data(), n * 4, hipMemcpyHostToDevice));
  const dim3 blk(T, T), grid((nx + T - 1) / T, (ny + T - 1) / T);
  for (int s = 0; s < steps; ++s) {
    calculate_temp<<<grid, blk>>>(p, s % 2 ? t1 : t0, s % 2 ? t0 : t1, nx, ny, 0.05f, 0.1f, 0.1f, 0.01f, 300.f);
    APP_HIP(hipGetLastError());
  }
  APP_HIP(hipDeviceSynchronize());
  APP_HIP(hipMemcpy(ht.data(), steps % 2 ? t1 : t0, n * 4, hipMemcpyDeviceToHost));
  double sum = 0;
  for (size_t i = 0; i < n; ++i) sum += ht[i];
  const bool ok = std::isfinite(sum) && sum / n > 300 && sum / n < 400;
  printf("hotspot %dx%d steps=%d: mean %.4f %s\n", nx, ny, steps, sum / n, ok ? "PASSED" : "FAILED");
  APP_HIP(hipFree(p));
  APP_HIP(hipFree(t0));
  APP_HIP(hipFree(t1));
  return ok ? 0 : 1;
}
