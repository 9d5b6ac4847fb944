// vectorAdd (the reference's tracer test app, nvbit_release/test-apps/vectoradd:
// c = a + b over doubles, 1024-thread blocks), plain HIP.
#include <cmath>

#include "app_common.h"

__global__ void vecAdd(const double* a, const double* b, double* c, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1 << 20;
  std::vector<double> ha(n), hb(n), hc(n);
  for (int i = 0; i < n; ++i) {
    ha[i] = std::sin((double)i) * std::sin((double)i);
    hb[i] = std::cos((double)i) * std::cos((double)i);
  }
  double *a, *b, *c;
  APP_HIP(hipMalloc(&a, n * sizeof(double)));
  APP_HIP(hipMalloc(&b, n * sizeof(double)));
  APP_HIP(hipMalloc(&c, n * sizeof(double)));
  APP_HIP(hipMemcpy(a, ha.data(), n * sizeof(double), hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(b, hb.data(), n * sizeof(double), hipMemcpyHostToDevice));
  const int block = 1024, grid = (n + block - 1) / block;
  vecAdd<<<grid, block>>>(a, b, c, n);
  APP_HIP(hipGetLastError());
  APP_HIP(hipDeviceSynchronize());
  APP_HIP(hipMemcpy(hc.data(), c, n * sizeof(double), hipMemcpyDeviceToHost));
  double sum = 0;
  for (int i = 0; i < n; ++i) sum += hc[i];
  const bool ok = std::fabs(sum / n - 1.0) < 1e-9;
  printf("vectoradd n=%d: result %.9f %s\n", n, sum / n, ok ? "PASSED" : "FAILED");
  APP_HIP(hipFree(a));
  APP_HIP(hipFree(b));
  APP_HIP(hipFree(c));
  return ok ? 0 : 1;
}
