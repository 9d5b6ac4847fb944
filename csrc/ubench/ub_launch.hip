// Kernel launch latency as the correlator sees it (reference
// GPU_Microbenchmark/ubench/system/kernel_lat: kernel_lat_{1..2048}TB).
//
// The correlator turns a kernel's rocprofv3 duration (End - Start timestamp)
// into hardware cycles, so the simulator's -gpgpu_kernel_launch_latency and
// -gpgpu_TB_launch_latency must be the fixed and per-workgroup parts of THAT
// duration, not of host-side launch throughput.  This program only launches
// isolated empty kernels (one per grid size, synchronised, 40 repetitions);
// run it under `rocprofv3 --kernel-trace` and fit the durations with
// accel_sim_framework_distributed_amd/hw_stats/launch_latency.py.  Run
// standalone it prints host-side event timings of the same launches.
#include <chrono>

#include "ubench.h"

__global__ void ub_empty_kernel(int* sink) {
  if (sink && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 1;
}

__global__ void ub_empty_queued(int* sink) {
  if (sink && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 2;
}

__global__ void ub_empty_idle(int* sink) {
  if (sink && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 3;
}

__global__ void ub_empty_chain(int* sink) {
  if (sink && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 4;
}

// reads one word per 4 KB page of a buffer the host just copied in
__global__ void ub_touch_after_copy(const int* __restrict__ buf, size_t pages, int* sink) {
  int acc = 0;
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < pages; p += (size_t)gridDim.x * blockDim.x)
    acc += buf[p * 1024];
  if (acc == 0x7fffffff) sink[0] = acc;
}
__global__ void ub_touch_again(const int* __restrict__ buf, size_t pages, int* sink) {
  int acc = 0;
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < pages; p += (size_t)gridDim.x * blockDim.x)
    acc += buf[p * 1024];
  if (acc == 0x7fffffff) sink[0] = acc + 1;
}

static void host_spin_us(double us) {
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < us) {
  }
}

// keeps the GPU busy (and its clocks up) for ~20 us before each measured launch,
// like the kernel a real application launched just before
__global__ void ub_warm_kernel(int spin, float* sink) {
  float x = (float)threadIdx.x;
  for (int i = 0; i < spin; ++i) x = __builtin_fmaf(x, 1.0000001f, 0.5f);
  if (x == -1.0f) sink[0] = x;
}

int main() {
  UbDevice dev;
  const double mhz = ub_shader_mhz();
  printf("device %s, %d CUs\n", dev.p.gcnArchName, dev.cus());
  printf("# measured_shader_mhz %.1f\n", mhz);
  UbTimer t;
  const int grids[] = {1, 16, 64, 256, 1024, 4096, 16384};
  for (int nb : grids) {
    double best = 1e30;
    for (int r = 0; r < 40; ++r) {
      hipLaunchKernelGGL(ub_warm_kernel, dim3(256), dim3(64), 0, 0, 20000, nullptr);
      t.start();
      hipLaunchKernelGGL(ub_empty_kernel, dim3(nb), dim3(64), 0, 0, nullptr);
      const double us = t.stop_ms() * 1e3;
      best = std::min(best, us);
      UB_CHECK(hipDeviceSynchronize());
    }
    printf("empty kernel, %5d workgroups: best event time %.2f us\n", nb, best);
  }
  // queued launches: empty kernels issued back to back behind a busy kernel,
  // with no event or synchronisation in between -- how an application's
  // consecutive kernels reach the GPU (rocprofv3 durations of these give the
  // per-kernel cost of a queued launch, -gpgpu_kernel_launch_latency_queued)
  for (int nb : {1, 64, 1024}) {
    for (int r = 0; r < 10; ++r) {
      hipLaunchKernelGGL(ub_warm_kernel, dim3(256), dim3(64), 0, 0, 20000, nullptr);
      for (int q = 0; q < 8; ++q) hipLaunchKernelGGL(ub_empty_queued, dim3(nb), dim3(64), 0, 0, nullptr);
      UB_CHECK(hipDeviceSynchronize());
    }
    printf("queued empty kernels, %5d workgroups: launched\n", nb);
  }
  // idle launches: the queue is empty and the GPU idle when the kernel is
  // submitted (no event, a host gap after the previous synchronisation) --
  // how a host-bound application loop (pathfinder, nw) reaches the GPU
  for (int nb : {1, 64, 1024, 4096}) {
    for (int r = 0; r < 30; ++r) {
      UB_CHECK(hipDeviceSynchronize());
      host_spin_us(30.0);
      hipLaunchKernelGGL(ub_empty_idle, dim3(nb), dim3(64), 0, 0, nullptr);
    }
    UB_CHECK(hipDeviceSynchronize());
    printf("idle empty kernels, %5d workgroups: launched\n", nb);
  }
  // chains: 64 empty kernels submitted back to back from an idle GPU; the
  // start-to-start interval in steady state is the host submission interval
  // (or the GPU's per-kernel throughput, whichever is longer)
  for (int r = 0; r < 4; ++r) {
    UB_CHECK(hipDeviceSynchronize());
    host_spin_us(30.0);
    for (int q = 0; q < 64; ++q) hipLaunchKernelGGL(ub_empty_chain, dim3(64), dim3(64), 0, 0, nullptr);
  }
  UB_CHECK(hipDeviceSynchronize());
  printf("chained empty kernels: launched\n");
  // first kernel after a host-to-device copy vs the same kernel again: what
  // the copy (and the first touch of its pages) adds to a kernel's duration
  {
    const size_t bytes = size_t(8) << 20, pages = bytes / 4096;
    std::vector<int> h(bytes / 4, 1);
    int* d = nullptr;
    UB_CHECK(hipMalloc(&d, bytes));
    for (int r = 0; r < 20; ++r) {
      UB_CHECK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
      hipLaunchKernelGGL(ub_touch_after_copy, dim3(64), dim3(64), 0, 0, d, pages, nullptr);
      UB_CHECK(hipDeviceSynchronize());
      host_spin_us(30.0);
      hipLaunchKernelGGL(ub_touch_again, dim3(64), dim3(64), 0, 0, d, pages, nullptr);
      UB_CHECK(hipDeviceSynchronize());
    }
    UB_CHECK(hipFree(d));
    printf("after-copy kernels: launched\n");
  }
  return 0;
}
