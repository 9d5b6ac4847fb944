// Device-function calls, plain HIP: the kernel calls non-inlined device
// functions (s_getpc_b64 / s_swappc_b64 / s_setpc_b64 return), one of which
// loops over a __constant__ table, and reads a __device__ variable -- the
// control flow and PC-relative addressing of library kernels such as RCCL's
// generic kernel, at test size (isatrace: device functions are instrumented
// with the kernel's probe window; tests/test_isatrace.py).
#include <cmath>

#include "app_common.h"

__constant__ float c_tab[16] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__device__ float g_bias[64];

__device__ __noinline__ float dev_poly(float x, const float* t, int k) {
  float acc = 0.f;
  for (int i = 0; i < k; ++i) acc = acc * x + t[i] * c_tab[i & 15];
  return acc;
}

__device__ __noinline__ float dev_root(float x) { return sqrtf(fabsf(x)) + 1.0f; }

__global__ void devcalls(const float* in, const float* t, float* out, int n, int k) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = in[i];
  const float y = (i & 1) ? dev_poly(x, t, k) : dev_root(x);
  out[i] = y + g_bias[i & 63];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, k = 8;
  std::vector<float> hin(n), ht(k), hb(64), hout(n);
  for (int i = 0; i < n; ++i) hin[i] = 0.001f * (float)(i % 997) - 0.3f;
  for (int i = 0; i < k; ++i) ht[i] = 0.5f + 0.25f * (float)i;
  for (int i = 0; i < 64; ++i) hb[i] = 0.01f * (float)i;
  float *in, *t, *out;
  APP_HIP(hipMalloc(&in, n * sizeof(float)));
  APP_HIP(hipMalloc(&t, k * sizeof(float)));
  APP_HIP(hipMalloc(&out, n * sizeof(float)));
  APP_HIP(hipMemcpy(in, hin.data(), n * sizeof(float), hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(t, ht.data(), k * sizeof(float), hipMemcpyHostToDevice));
  APP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_bias), hb.data(), sizeof(hb[0]) * 64));
  devcalls<<<(n + 255) / 256, 256>>>(in, t, out, n, k);
  APP_HIP(hipGetLastError());
  APP_HIP(hipDeviceSynchronize());
  APP_HIP(hipMemcpy(hout.data(), out, n * sizeof(float), hipMemcpyDeviceToHost));
  const float ctab[16] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    float y;
    if (i & 1) {
      float acc = 0.f;
      for (int j = 0; j < k; ++j) acc = acc * hin[i] + ht[j] * ctab[j & 15];
      y = acc;
    } else {
      y = std::sqrt(std::fabs(hin[i])) + 1.0f;
    }
    y += hb[i & 63];
    if (std::fabs(y - hout[i]) > 1e-3f * (1.0f + std::fabs(y))) ++bad;
  }
  printf("devcalls n=%d: %d mismatches %s\n", n, bad, bad ? "FAILED" : "PASSED");
  APP_HIP(hipFree(in));
  APP_HIP(hipFree(t));
  APP_HIP(hipFree(out));
  return bad ? 1 : 0;
}
