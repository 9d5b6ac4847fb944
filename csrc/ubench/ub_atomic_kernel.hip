// Atomics and launch overheads (reference GPU_Microbenchmark
// atomics/Atomic_add_{bw,bw_conflict,lat} and system/kernel_lat):
//  * global atomicAdd latency (dependent chain, one lane),
//  * throughput without conflicts (every lane its own word) and with full
//    conflicts (every lane of the chip on one word),
//  * empty-kernel launch latency vs number of workgroups, fitted to
//    kernel_launch_latency + n_blocks * tb_launch_latency.
#include "ubench.h"

__global__ void atom_lat(unsigned* p, int iters, uint64_t* out) {
  if (threadIdx.x) return;
  unsigned v = 0;
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) v = atomicAdd(p + (v & 0), 1u);
  uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = v;
}

__global__ void atom_bw(unsigned* p, int iters, int conflict) {
  unsigned* q = conflict ? p : p + blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < iters; ++i) atomicAdd(q, 1u);
}

__global__ void empty_kernel() {}

int main() {
  UbDevice d;
  const int cus = d.cus();
  unsigned* p;
  uint64_t* o;
  const int blocks = cus * 8, threads = 256;
  UB_CHECK(hipMalloc(&p, (size_t)blocks * threads * 4));
  UB_CHECK(hipMemset(p, 0, (size_t)blocks * threads * 4));
  UB_CHECK(hipMalloc(&o, 16));
  const int iters = 2048;
  hipLaunchKernelGGL(atom_lat, dim3(1), dim3(64), 0, 0, p, iters, o);
  uint64_t h[2];
  UB_CHECK(hipMemcpy(h, o, 16, hipMemcpyDeviceToHost));
  const double lat = (double)h[0] / iters;
  UbTimer t;
  double rate[2];
  for (int c = 0; c < 2; ++c) {
    const int it = c ? 16 : 256;
    hipLaunchKernelGGL(atom_bw, dim3(blocks), dim3(threads), 0, 0, p, it, c);
    UB_CHECK(hipDeviceSynchronize());
    t.start();
    hipLaunchKernelGGL(atom_bw, dim3(blocks), dim3(threads), 0, 0, p, it, c);
    rate[c] = (double)blocks * threads * it / (t.stop_ms() * 1e-3) / 1e9;
  }
  printf("atomicAdd latency %.1f cycles; %.2f G atomics/s distinct, %.3f G atomics/s same-address\n", lat, rate[0],
         rate[1]);
  // launch latency: time 200 back-to-back empty launches for each grid size
  std::vector<std::pair<double, double>> pts;
  for (int nb : {1, 64, 256, 1024, 4096, 16384}) {
    hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(64), 0, 0);
    UB_CHECK(hipDeviceSynchronize());
    t.start();
    for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(64), 0, 0);
    const double us = t.stop_ms() * 1e3 / 200;
    pts.push_back({(double)nb, us});
    printf("empty kernel, %5d workgroups: %.2f us/launch\n", nb, us);
  }
  // least squares us = a + b * nb
  double sx = 0, sy = 0, sxx = 0, sxy = 0;
  for (auto& q : pts) {
    sx += q.first;
    sy += q.second;
    sxx += q.first * q.first;
    sxy += q.first * q.second;
  }
  const double n = (double)pts.size();
  const double b = (n * sxy - sx * sy) / (n * sxx - sx * sx), a = (sy - b * sx) / n;
  const double mhz = ub_shader_mhz();
  printf("# launch_us %.3f  per_block_us %.5f  shader_mhz %.0f\n", a, b, mhz);
  // launch overhead between back-to-back kernels is host/CP time that a
  // kernel's own (rocprofv3 start..end) duration does not contain: it is
  // reported, while the simulated kernel starts issuing at once; the
  // per-workgroup slope is the dispatcher cost per CTA
  printf("# kernel_launch_overhead_cycles %.0f\n", a * mhz);
  // the simulator's launch latencies are fitted to rocprofv3 durations of
  // isolated empty kernels instead (ub_launch + hw_stats/launch_latency.py)
  UB_CHECK(hipFree(p));
  UB_CHECK(hipFree(o));
  return 0;
}
