// hotspot-shaped thermal stencil (Rodinia hotspot: 2-D grid of temperatures
// + power map, 5-point update per step, 16x16 tiles staged through shared
// memory), HIP + asim_trace annotations.  One launch per simulated step,
// ping-ponging between two temperature buffers.
#include <cmath>

#include "../tracer/asim_trace.h"

using namespace asim_trace;

constexpr int T = 16;

template <class TR>
__global__ void calculate_temp(TR tr, const float* power, const float* tin, float* tout, int nx, int ny, float cap,
                               float rx, float ry, float rz, float amb) {
  __shared__ float tile[T + 2][T + 2];
  auto w = tr.wave();
  const int gx = blockIdx.x * T + threadIdx.x, gy = blockIdx.y * T + threadIdx.y;
  const int tx = threadIdx.x + 1, ty = threadIdx.y + 1;
  ASIM_VALU(w, V_MAD_U32_U24, 1, 0);
  ASIM_VALU(w, V_MAD_U32_U24, 2, 0);
  ASIM_VALU(w, V_MAD_U32_U24, 3, 1, 2);  // linear index
  const bool in = gx < nx && gy < ny;
  const int idx = gy * nx + gx;
  float c = 0.f;
  if (in) c = ASIM_LD(w, GLOBAL_LOAD_DWORD, tin + idx, 4, 3);
  ASIM_VALU(w, S_WAITCNT, 0, 0);
  ASIM_ST(w, DS_WRITE_B32, &tile[ty][tx], c, 4, 5);
  // halo: edge threads fetch the neighbour tile's border (clamped at the grid edge)
  if (threadIdx.x == 0) {
    const int hx = gx > 0 ? gx - 1 : gx;
    float v = 0.f;
    if (gy < ny) v = ASIM_LD(w, GLOBAL_LOAD_DWORD, tin + gy * nx + hx, 6, 3);
    ASIM_ST(w, DS_WRITE_B32, &tile[ty][0], v, 6, 5);
  }
  if (threadIdx.x == T - 1) {
    const int hx = gx + 1 < nx ? gx + 1 : gx;
    float v = 0.f;
    if (gy < ny) v = ASIM_LD(w, GLOBAL_LOAD_DWORD, tin + gy * nx + hx, 6, 3);
    ASIM_ST(w, DS_WRITE_B32, &tile[ty][T + 1], v, 6, 5);
  }
  if (threadIdx.y == 0) {
    const int hy = gy > 0 ? gy - 1 : gy;
    float v = 0.f;
    if (gx < nx) v = ASIM_LD(w, GLOBAL_LOAD_DWORD, tin + hy * nx + gx, 7, 3);
    ASIM_ST(w, DS_WRITE_B32, &tile[0][tx], v, 7, 5);
  }
  if (threadIdx.y == T - 1) {
    const int hy = gy + 1 < ny ? gy + 1 : gy;
    float v = 0.f;
    if (gx < nx) v = ASIM_LD(w, GLOBAL_LOAD_DWORD, tin + hy * nx + gx, 7, 3);
    ASIM_ST(w, DS_WRITE_B32, &tile[T + 1][tx], v, 7, 5);
  }
  ASIM_BARRIER(w);
  if (in) {
    const float p = ASIM_LD(w, GLOBAL_LOAD_DWORD, power + idx, 8, 3);
    const float n_ = ASIM_LD(w, DS_READ_B32, &tile[ty - 1][tx], 9, 5);
    const float s_ = ASIM_LD(w, DS_READ_B32, &tile[ty + 1][tx], 10, 5);
    const float e_ = ASIM_LD(w, DS_READ_B32, &tile[ty][tx + 1], 11, 5);
    const float w_ = ASIM_LD(w, DS_READ_B32, &tile[ty][tx - 1], 12, 5);
    ASIM_VALU(w, S_WAITCNT, 0, 0);
    ASIM_VALU(w, V_ADD_F32, 13, 9, 10);
    ASIM_VALU(w, V_FMA_F32, 13, 4, 13);
    ASIM_VALU(w, V_ADD_F32, 14, 11, 12);
    ASIM_VALU(w, V_FMA_F32, 14, 4, 14);
    ASIM_VALU(w, V_FMA_F32, 15, 13, 14, 8);
    ASIM_VALU(w, V_FMA_F32, 15, 4, 15);
    ASIM_VALU(w, V_FMA_F32, 16, 15, 4);
    const float d = cap * (p + (s_ + n_ - 2.f * c) * ry + (e_ + w_ - 2.f * c) * rx + (amb - c) * rz);
    ASIM_ST(w, GLOBAL_STORE_DWORD, tout + idx, c + d, 16, 3);
  }
  w.exit();
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
  ASIM_HIP(hipMalloc(&p, n * 4));
  ASIM_HIP(hipMalloc(&t0, n * 4));
  ASIM_HIP(hipMalloc(&t1, n * 4));
  memcpy_htod(p, hp.data(), n * 4);
  memcpy_htod(t0, ht.data(), n * 4);
  const dim3 blk(T, T), grid((nx + T - 1) / T, (ny + T - 1) / T);
  for (int s = 0; s < steps; ++s) {
    launch("_Z14calculate_tempPfS_S_iiffff", calculate_temp<On>, calculate_temp<Off>, grid, blk, 0, 0,
           (const float*)p, (const float*)(s % 2 ? t1 : t0), s % 2 ? t0 : t1, nx, ny, 0.05f, 0.1f, 0.1f, 0.01f, 300.f);
  }
  ASIM_HIP(hipDeviceSynchronize());
  ASIM_HIP(hipMemcpy(ht.data(), steps % 2 ? t1 : t0, n * 4, hipMemcpyDeviceToHost));
  double sum = 0;
  for (size_t i = 0; i < n; ++i) sum += ht[i];
  const bool ok = std::isfinite(sum) && sum / n > 300 && sum / n < 400;
  printf("hotspot %dx%d steps=%d: mean %.4f %s\n", nx, ny, steps, sum / n, ok ? "PASSED" : "FAILED");
  ASIM_HIP(hipFree(p));
  ASIM_HIP(hipFree(t0));
  ASIM_HIP(hipFree(t1));
  return ok ? 0 : 1;
}
