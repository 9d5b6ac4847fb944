// Peak arithmetic throughput per data type and the register-file bandwidth
// it implies (reference GPU_Microbenchmark core/MaxFlops_{double,float,int32}, core/config_{dpu,fpu,int} and core/regfile_bw): every CU runs 8
// waves of independent FMA chains (8 accumulators per lane, no dependency
// between consecutive instructions), timed with hipEvents over the grid.
// Prints TFLOP/s (TOP/s for int32), operations per CU per shader cycle, and
// the lanes-per-cycle figure the tuner's unit counts correspond to.
#include "ubench.h"

template <class T>
__device__ __forceinline__ T fma_op(T a, T b, T c) { return a * b + c; }

template <class T, int ITERS>
__global__ void ub_flops_kernel(T seed, T m, T c, T* sink) {
  // m, c are kernel arguments: the compiler cannot fold the FMA chains
  T a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = seed + (T)(threadIdx.x + k);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fma_op(a[k], m, c);
  }
  T s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  if (s == (T)-12345) sink[0] = s;  // keeps the chains alive
}

template <class F>
static double timed_ms(F launch) {
  launch();
  UB_CHECK(hipDeviceSynchronize());
  UbTimer t;
  t.start();
  for (int r = 0; r < 5; ++r) launch();
  return t.stop_ms() / 5.0;
}

int main() {
  UbDevice d;
  const int cus = d.cus(), waves = 8, threads = 64 * waves;
  const double mhz = ub_shader_mhz();
  printf("# measured_shader_mhz %.1f\n", mhz);
  void* sink;
  UB_CHECK(hipMalloc(&sink, 64));
  const dim3 grid(cus * 4), block(threads);
  const double lanes = (double)grid.x * threads;
  struct Row { const char* name; double ms; double ops_per_lane; };
  std::vector<Row> rows;
  rows.push_back({"fp64 (v_fma_f64)", timed_ms([&] {
                    hipLaunchKernelGGL((ub_flops_kernel<double, 2048>), grid, block, 0, 0, 1.0, 1.0001, 0.5, (double*)sink); }),
                  2.0 * 8 * 2048});
  rows.push_back({"fp32 (v_fma_f32)", timed_ms([&] {
                    hipLaunchKernelGGL((ub_flops_kernel<float, 4096>), grid, block, 0, 0, 1.f, 1.0001f, 0.5f, (float*)sink); }),
                  2.0 * 8 * 4096});
  rows.push_back({"int32 (v_mad_u32)", timed_ms([&] {
                    hipLaunchKernelGGL((ub_flops_kernel<uint32_t, 4096>), grid, block, 0, 0, 1u, 3u, 7u, (uint32_t*)sink); }),
                  2.0 * 8 * 4096});
  for (const Row& r : rows) {
    const double ops = lanes * r.ops_per_lane;
    const double tops = ops / (r.ms * 1e-3) / 1e12;
    const double per_cu_cycle = ops / (r.ms * 1e-3) / (mhz * 1e6) / cus;
    printf("%-24s %8.2f T(FL)OP/s  %7.1f ops/CU/cycle\n", r.name, tops, per_cu_cycle);
  }
  // register-file read bandwidth of the fp32 FMA stream: 3 operands x 4 B per lane op
  const double fp32_lane_ops = rows[1].ops_per_lane / 2.0 * lanes / (rows[1].ms * 1e-3);
  printf("# regfile_read_TBps %.1f\n", fp32_lane_ops * 12.0 / 1e12);
  printf("# fp32_lanes_per_cu_cycle %.1f\n", fp32_lane_ops / (mhz * 1e6) / cus);
  UB_CHECK(hipFree(sink));
  return 0;
}
