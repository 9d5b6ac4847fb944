// Vector-L1 data path under strided lane addresses (no reference counterpart:
// GPGPU-Sim's L1 moves whole lines; the fitted MI355X data path of
// -sim_l1_port_bytes is measured with dense loads in ub_bw_widths).
//
// Every workgroup re-reads an L1-resident 16 KB region with 4-byte loads
// whose lanes are `stride` bytes apart (4 = dense ... 128 = one lane per
// line): the wave-load rate per CU tells what the data stage moves per line
// an access touches -- the bytes the lanes use, whole 32 B sectors or whole
// 64 B halves (the simulator's -sim_l1_port_granule 0 / 32 / 64).
#include "ubench.h"

__global__ void __launch_bounds__(256) l1s_read(const float* __restrict__ a, int stride_f, int reps, float* sink) {
  // region: 16 KB = 4096 floats, shared by the workgroup's 4 waves
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0;
  for (int r = 0; r < reps; ++r) {
    // each wave-load covers 64 * stride bytes; successive loads walk the region
    const int idx = ((r * 4 + wave) * 64 * stride_f + lane * stride_f) & 4095;
    acc += a[idx];
  }
  if (acc == -1.f) sink[0] = acc;
}

int main() {
  UbDevice d;
  const double mhz = ub_shader_mhz();
  const int cus = d.cus();
  float *buf, *sink;
  UB_CHECK(hipMalloc(&buf, 16384));
  UB_CHECK(hipMalloc(&sink, 4));
  UB_CHECK(hipMemset(buf, 0, 16384));
  printf("device %s, %d CUs, %.0f MHz\n", d.p.gcnArchName, cus, mhz);
  printf("%8s %12s %14s %16s\n", "stride", "lines/load", "cycles/load", "used B/clk/CU");
  const int blocks = cus * 4, reps = 4096;
  double dense = 0;
  for (int stride : {4, 8, 16, 32, 64, 128}) {
    const int sf = stride / 4;
    hipLaunchKernelGGL(l1s_read, dim3(blocks), dim3(256), 0, 0, buf, sf, 8, sink);  // warm
    UB_CHECK(hipDeviceSynchronize());
    std::vector<double> v;
    for (int rep = 0; rep < 5; ++rep) {
      UbTimer t;
      t.start();
      hipLaunchKernelGGL(l1s_read, dim3(blocks), dim3(256), 0, 0, buf, sf, reps, sink);
      v.push_back(t.stop_ms());
    }
    std::sort(v.begin(), v.end());
    const double cyc = v[2] * 1e-3 * mhz * 1e6;
    const double loads_per_cu = (double)blocks / cus * 4 * reps;  // wave-loads per CU
    const double cpl = cyc / loads_per_cu;
    const int lines = std::max(1, 64 * stride / 128);
    if (stride == 4) dense = cpl;
    printf("%8d %12d %14.2f %16.2f\n", stride, lines, cpl, 256.0 / cpl);
    printf("# l1_stride_%d_cycles_per_load %.2f\n", stride, cpl);
  }
  printf("# l1_stride_dense_cycles_per_load %.2f\n", dense);
  UB_CHECK(hipFree(buf));
  UB_CHECK(hipFree(sink));
  return 0;
}
