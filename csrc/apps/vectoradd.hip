// vectorAdd (the reference's tracer test app, nvbit_release/test-apps/vectoradd:
// c = a + b over doubles, 1024-thread blocks), written for trace capture on
// MI355X with asim_trace annotations that follow the gfx950 ISA of the plain
// build (address calc, two 8-byte loads, waitcnt, v_add_f64, 8-byte store).
#include <cmath>

#include "../tracer/asim_trace.h"

using namespace asim_trace;

template <class TR>
__global__ void vecAdd(TR tr, const double* a, const double* b, double* c, int n) {
  auto w = tr.wave();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  ASIM_VALU(w, S_MUL_I32, 0, 0);
  ASIM_VALU(w, V_ADD_U32, 1, 0);
  ASIM_VALU(w, V_CMP_GT_I32, 0, 1);
  if (i < n) {
    ASIM_VALU(w, V_LSHLREV_B32, 2, 1);
    const double x = ASIM_LD(w, GLOBAL_LOAD_DWORDX2, a + i, 3, 2);
    const double y = ASIM_LD(w, GLOBAL_LOAD_DWORDX2, b + i, 4, 2);
    ASIM_VALU(w, S_WAITCNT, 0, 0);
    ASIM_VALU(w, V_ADD_F64, 5, 3, 4);
    ASIM_ST(w, GLOBAL_STORE_DWORDX2, c + i, x + y, 5, 2);
  }
  w.exit();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1 << 20;
  std::vector<double> ha(n), hb(n), hc(n);
  for (int i = 0; i < n; ++i) {
    ha[i] = std::sin((double)i) * std::sin((double)i);
    hb[i] = std::cos((double)i) * std::cos((double)i);
  }
  double *a, *b, *c;
  ASIM_HIP(hipMalloc(&a, n * sizeof(double)));
  ASIM_HIP(hipMalloc(&b, n * sizeof(double)));
  ASIM_HIP(hipMalloc(&c, n * sizeof(double)));
  memcpy_htod(a, ha.data(), n * sizeof(double));
  memcpy_htod(b, hb.data(), n * sizeof(double));
  const int block = 1024, grid = (n + block - 1) / block;
  launch("_Z6vecAddPdS_S_i", vecAdd<On>, vecAdd<Off>, dim3(grid), dim3(block), 0, 0, (const double*)a,
         (const double*)b, c, n);
  ASIM_HIP(hipDeviceSynchronize());
  ASIM_HIP(hipMemcpy(hc.data(), c, n * sizeof(double), hipMemcpyDeviceToHost));
  double sum = 0;
  for (int i = 0; i < n; ++i) sum += hc[i];
  const bool ok = std::fabs(sum / n - 1.0) < 1e-9;
  printf("vectoradd n=%d: result %.9f %s\n", n, sum / n, ok ? "PASSED" : "FAILED");
  ASIM_HIP(hipFree(a));
  ASIM_HIP(hipFree(b));
  ASIM_HIP(hipFree(c));
  return ok ? 0 : 1;
}
