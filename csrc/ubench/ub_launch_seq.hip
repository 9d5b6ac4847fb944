// What a kernel's rocprofv3 duration contains when it runs right behind
// another one, after a copy, in a chain, or after a host gap (no reference
// counterpart: the reference's kernel_lat measures isolated launches and
// GPGPU-Sim charges every kernel the same -gpgpu_kernel_launch_latency).
//
// Every kernel stamps, on the device's 100 MHz constant clock
// (s_memrealtime), the first wave's start and the last wave's end of its
// launch, and each wave busy-waits a given time from its own start: the
// launch's execution window is known on the device independently of the
// rocprofv3 timestamps.  Run under
//   rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -- ub_launch_seq
// and read with accel_sim_framework_distributed_amd/hw_stats/launch_seq.py:
// per scenario the rocprofv3 duration, the device execution window, the
// device gap to the previous kernel and the host submission times give the
// launch model's terms (idle launch, queued dispatch gap, the part of a
// queued duration spent behind the previous kernel, the host interval).
//
// Scenarios (kernel names say which; launch ids are dispatch order):
//   ls_idle   sync, 30 us host gap, one kernel (W = 0 / 3 us)
//   ls_pair_a / ls_pair_b   A (T = 0 / 4 / 12 / 30 us) then B (W = 0 / 3 us)
//             queued right behind it
//   ls_chain  24 kernels of W = 0 / 1 / 3 / 8 us submitted back to back
//   ls_gap    kernels of 3 us submitted with a host gap G = 2 / 5 / 10 / 20 us
//   ls_copy_k / ls_copy_k2  the bfs loop: H2D 4 B, kernel (3 us), kernel
//             (1 us) queued behind it, D2H 4 B
//   ls_d2h_k  the srad loop: kernel, kernel, D2H 64 KB, next pair
#include <chrono>

#include "ubench.h"

struct Stamps {
  unsigned long long* ts;  // first wave start per launch id (init ~0)
  unsigned long long* te;  // last wave end per launch id (init 0)
};

__device__ __forceinline__ void ls_body(uint64_t ticks, uint32_t id, Stamps s) {
  if ((threadIdx.x & 63) != 0) return;
  const uint64_t t0 = ub_realtime();
  atomicMin(&s.ts[id], (unsigned long long)t0);
  uint64_t t = t0;
  while (t - t0 < ticks) t = ub_realtime();
  atomicMax(&s.te[id], (unsigned long long)t);
}

#define LS_KERNEL(name) \
  __global__ void name(uint64_t ticks, uint32_t id, Stamps s) { ls_body(ticks, id, s); }
LS_KERNEL(ls_idle)
LS_KERNEL(ls_pair_a)
LS_KERNEL(ls_pair_b)
LS_KERNEL(ls_chain)
LS_KERNEL(ls_gap)
LS_KERNEL(ls_copy_k)
LS_KERNEL(ls_copy_k2)
LS_KERNEL(ls_d2h_k)

static void host_spin_us(double us) {
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < us) {
  }
}

static constexpr uint32_t kMaxLaunch = 4096;
static constexpr int kGrid = 256, kBlock = 64;

int main() {
  UbDevice dev;
  const double mhz = ub_shader_mhz();
  printf("device %s, %d CUs\n", dev.p.gcnArchName, dev.cus());
  printf("# measured_shader_mhz %.1f\n", mhz);
  Stamps s;
  UB_CHECK(hipMalloc(&s.ts, kMaxLaunch * sizeof(unsigned long long)));
  UB_CHECK(hipMalloc(&s.te, kMaxLaunch * sizeof(unsigned long long)));
  UB_CHECK(hipMemset(s.ts, 0xff, kMaxLaunch * sizeof(unsigned long long)));
  UB_CHECK(hipMemset(s.te, 0, kMaxLaunch * sizeof(unsigned long long)));
  int* d4 = nullptr;
  char* d64k = nullptr;
  UB_CHECK(hipMalloc(&d4, 4));
  UB_CHECK(hipMalloc(&d64k, 65536));
  std::vector<char> h64k(65536, 0);
  int h4 = 0;
  UB_CHECK(hipDeviceSynchronize());
  uint32_t id = 0;
  auto us = [](double u) { return (uint64_t)(u * 100.0); };  // 100 MHz ticks
  auto launch = [&](void (*k)(uint64_t, uint32_t, Stamps), double work_us, const char* tag) {
    if (id >= kMaxLaunch) {
      fprintf(stderr, "too many launches\n");
      exit(3);
    }
    hipLaunchKernelGGL(k, dim3(kGrid), dim3(kBlock), 0, 0, us(work_us), id, s);
    printf("L %u %s %.1f\n", id, tag, work_us);
    ++id;
  };
  auto settle = [&] {
    UB_CHECK(hipDeviceSynchronize());
    host_spin_us(30.0);
  };
  // warm the clocks up with a ~2 ms busy kernel
  hipLaunchKernelGGL(ls_idle, dim3(kGrid), dim3(kBlock), 0, 0, us(2000.0), kMaxLaunch - 1, s);
  UB_CHECK(hipDeviceSynchronize());
  for (double w : {0.0, 3.0})
    for (int r = 0; r < 10; ++r) {
      settle();
      launch(ls_idle, w, "idle");
    }
  for (double ta : {0.0, 4.0, 12.0, 30.0})
    for (double w : {0.0, 3.0})
      for (int r = 0; r < 8; ++r) {
        settle();
        launch(ls_pair_a, ta, "pair_a");
        launch(ls_pair_b, w, "pair_b");
      }
  for (double w : {0.0, 1.0, 3.0, 8.0})
    for (int r = 0; r < 3; ++r) {
      settle();
      for (int q = 0; q < 24; ++q) launch(ls_chain, w, "chain");
    }
  for (double g : {2.0, 5.0, 10.0, 20.0}) {
    settle();
    for (int q = 0; q < 16; ++q) {
      launch(ls_gap, 3.0, "gap");
      host_spin_us(g);
    }
    printf("G %.1f\n", g);
  }
  settle();
  for (int r = 0; r < 10; ++r) {
    UB_CHECK(hipMemcpy(d4, &h4, 4, hipMemcpyHostToDevice));
    launch(ls_copy_k, 3.0, "copy_k");
    launch(ls_copy_k2, 1.0, "copy_k2");
    UB_CHECK(hipMemcpy(&h4, d4, 4, hipMemcpyDeviceToHost));
  }
  settle();
  for (int r = 0; r < 10; ++r) {
    launch(ls_d2h_k, 3.0, "d2h_k");
    launch(ls_d2h_k, 2.0, "d2h_k");
    UB_CHECK(hipMemcpy(h64k.data(), d64k, 65536, hipMemcpyDeviceToHost));
  }
  UB_CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> ts(id), te(id);
  UB_CHECK(hipMemcpy(ts.data(), s.ts, id * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  UB_CHECK(hipMemcpy(te.data(), s.te, id * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < id; ++i) printf("S %u %llu %llu\n", i, ts[i], te[i]);
  printf("launches %u\n", id);
  UB_CHECK(hipFree(s.ts));
  UB_CHECK(hipFree(s.te));
  UB_CHECK(hipFree(d4));
  UB_CHECK(hipFree(d64k));
  return 0;
}
