// nn-shaped nearest-neighbour distance kernel (Rodinia nn: Euclidean distance
// of every (lat, lng) record to a query point), HIP + asim_trace annotations.
#include <cmath>

#include "../tracer/asim_trace.h"

using namespace asim_trace;

template <class TR>
__global__ void euclid(TR tr, const float2* loc, float* dist, int n, float lat, float lng) {
  auto w = tr.wave();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  ASIM_VALU(w, V_MAD_U32_U24, 1, 0);
  ASIM_VALU(w, V_CMP_GT_I32, 0, 1);
  if (i < n) {
    ASIM_VALU(w, V_LSHLREV_B32, 2, 1);
    const float2 p = ASIM_LD(w, GLOBAL_LOAD_DWORDX2, loc + i, 3, 2);
    ASIM_VALU(w, S_WAITCNT, 0, 0);
    ASIM_VALU(w, V_ADD_F32, 4, 3);
    ASIM_VALU(w, V_ADD_F32, 5, 3);
    ASIM_VALU(w, V_MUL_F32, 6, 5, 5);
    ASIM_VALU(w, V_FMA_F32, 6, 4, 4, 6);
    ASIM_VALU(w, V_SQRT_F32, 7, 6);
    const float dx = lat - p.x, dy = lng - p.y;
    ASIM_ST(w, GLOBAL_STORE_DWORD, dist + i, sqrtf(dx * dx + dy * dy), 7, 2);
  }
  w.exit();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 42764 * 8;
  std::vector<float2> h(n);
  for (int i = 0; i < n; ++i) h[i] = make_float2(30.f + 10.f * std::sin(0.37f * i), 90.f * std::cos(0.11f * i));
  float2* d;
  float* dist;
  ASIM_HIP(hipMalloc(&d, n * sizeof(float2)));
  ASIM_HIP(hipMalloc(&dist, n * 4));
  memcpy_htod(d, h.data(), n * sizeof(float2));
  const int blk = 256;
  launch("_Z6euclidP7latLongPfiff", euclid<On>, euclid<Off>, dim3((n + blk - 1) / blk), dim3(blk), 0, 0,
         (const float2*)d, dist, n, 30.f, 90.f);
  ASIM_HIP(hipDeviceSynchronize());
  std::vector<float> out(n);
  ASIM_HIP(hipMemcpy(out.data(), dist, n * 4, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < n && ok; i += 997) {
    const float dx = 30.f - h[i].x, dy = 90.f - h[i].y;
    ok = std::fabs(out[i] - std::sqrt(dx * dx + dy * dy)) < 1e-3f;
  }
  printf("nn n=%d: %s\n", n, ok ? "PASSED" : "FAILED");
  ASIM_HIP(hipFree(d));
  ASIM_HIP(hipFree(dist));
  return ok ? 0 : 1;
}
