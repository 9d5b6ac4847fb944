// Cost of the LDS access patterns of the cycle engine's "uniform code on all
// 64 lanes" style (every lane reads / writes the same state word) on the
// MI355X it runs on: dependent read-modify-write chains of one 32/64-bit LDS
// word with all lanes active vs one lane active, and plain dependent reads.
// Prints shader clocks per chain step; no gpgpusim option (simulator cost).
#include "ubench.h"

template <int kMode>
__global__ void __launch_bounds__(64) ub_lds_chain(int iters, uint64_t* out, uint32_t* sink) {
  __shared__ uint64_t st[64];
  const int l = threadIdx.x;
  st[l] = l;
  __syncthreads();
  volatile uint64_t* v = st;
  const uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
    if (kMode == 0) {  // all lanes: read-modify-write of one 64-bit word
      v[3] = v[3] + 1;
    } else if (kMode == 1) {  // one lane performs the RMW
      if (l == 0) v[3] = v[3] + 1;
    } else if (kMode == 2) {  // all lanes: dependent reads (pointer chase in LDS)
      v[3] = v[(v[3] + 1) & 3];
    } else if (kMode == 3) {  // all lanes: 32-bit RMW
      volatile uint32_t* w = reinterpret_cast<volatile uint32_t*>(st);
      w[5] = w[5] + 1;
    }
  }
  const uint64_t t1 = ub_clock();
  if (l == 0) out[0] = t1 - t0;
  if (st[3] == 0xdeadbeef) sink[0] = 1;
}

template <int kMode>
static double run(int iters, uint64_t* d_out) {
  hipLaunchKernelGGL(ub_lds_chain<kMode>, dim3(1), dim3(64), 0, 0, iters, d_out, nullptr);
  UB_CHECK(hipDeviceSynchronize());
  uint64_t c = 0;
  UB_CHECK(hipMemcpy(&c, d_out, 8, hipMemcpyDeviceToHost));
  return (double)c / iters;
}

int main() {
  UbDevice dev;
  printf("device %s\n", dev.p.gcnArchName);
  uint64_t* d_out;
  UB_CHECK(hipMalloc(&d_out, 8));
  const int iters = 20000;
  run<0>(100, d_out);
  printf("LDS 64-bit RMW, all 64 lanes:   %.1f clocks/step\n", run<0>(iters, d_out));
  printf("LDS 64-bit RMW, one lane:       %.1f clocks/step\n", run<1>(iters, d_out));
  printf("LDS dependent read, all lanes:  %.1f clocks/step\n", run<2>(iters, d_out));
  printf("LDS 32-bit RMW, all 64 lanes:   %.1f clocks/step\n", run<3>(iters, d_out));
  return 0;
}
