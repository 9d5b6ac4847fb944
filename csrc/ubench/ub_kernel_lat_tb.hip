// Kernel duration against workgroup count (reference GPU_Microbenchmark
// system/kernel_lat, which times an empty kernel's launch; here the grid
// grows so the slope separates the per-workgroup dispatch cost from the
// fixed launch cost).  An empty kernel of 64-thread workgroups is launched
// back to back N times per size; the per-launch time against the grid size
// is fitted by least squares: intercept = fixed cost, slope = cost per
// workgroup of the whole-chip dispatcher (shader cycles).
// The simulator's launch model is pinned from rocprofv3 durations
// (hw_stats/launch_latency.py), so the fitted values print as suggestions.
#include "ubench.h"

__global__ void __launch_bounds__(64) empty_wg(int* sink) {
  if (threadIdx.x == 1000) sink[0] = 1;
}

int main() {
  UbDevice dev;
  const double mhz = ub_shader_mhz();
  printf("device %s, %d CUs, shader clock %.0f MHz\n", dev.p.gcnArchName, dev.cus(), mhz);
  int* sink;
  UB_CHECK(hipMalloc(&sink, 4));
  const int grids[] = {1, 256, 1024, 4096, 16384, 65536, 262144};
  const int reps = 200;
  std::vector<double> xs, ys;
  UbTimer t;
  for (int g : grids) {
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(empty_wg, dim3(g), dim3(64), 0, 0, sink);
    UB_CHECK(hipDeviceSynchronize());
    t.start();
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(empty_wg, dim3(g), dim3(64), 0, 0, sink);
    const double us = t.stop_ms() * 1000.0 / reps;
    printf("workgroups %7d: %9.3f us per kernel (%.4f us per 1k workgroups)\n", g, us, us / g * 1000.0);
    xs.push_back(g);
    ys.push_back(us);
  }
  // least squares over the grids large enough to be dispatch bound
  double sx = 0, sy = 0, sxx = 0, sxy = 0;
  int n = 0;
  for (size_t i = 0; i < xs.size(); ++i) {
    if (xs[i] < 1024) continue;
    sx += xs[i];
    sy += ys[i];
    sxx += xs[i] * xs[i];
    sxy += xs[i] * ys[i];
    ++n;
  }
  const double slope = (n * sxy - sx * sy) / (n * sxx - sx * sx);
  const double icpt = (sy - slope * sx) / n;
  const double per_wg_cycles = slope * mhz;
  printf("fit: %.3f us fixed + %.5f us per workgroup (%.2f shader cycles per workgroup, %.1f workgroups/cycle)\n",
         icpt, slope, per_wg_cycles, per_wg_cycles > 0 ? 1.0 / per_wg_cycles : 0.0);
  printf("# kernel_fixed_us %.3f\n# workgroup_dispatch_cycles %.3f\n# single_wg_kernel_us %.3f\n", icpt, per_wg_cycles,
         ys[0]);
  printf("# suggest_gpgpu_TB_launch_latency %d\n", (int)(per_wg_cycles + 0.5));
  UB_CHECK(hipFree(sink));
  return 0;
}
