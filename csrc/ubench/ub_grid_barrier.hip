// Price of one grid-wide barrier of the persistent cycle engine (its PDES
// epoch boundary, csrc/engine/grid_barrier.h) on the MI355X it runs on:
// blocks of one 64-lane wave, one per CU (the engine's LDS footprint), a
// fixed number of barriers per launch.  Variants: with / without the agent
// release+acquire fences, and with each wave publishing 2 KB of plain stores
// per epoch (the engine's outbox packets and counts) before arriving.
// Prints microseconds per barrier; no gpgpusim option (simulator-side cost).
#include "engine/grid_barrier.h"
#include "ubench.h"

using asim::GpuCtl;

template <bool kFence, int kStoreB>
__global__ void __launch_bounds__(64) ub_barrier_kernel(GpuCtl* ctl, uint32_t iters, uint4* box, uint64_t* cyc) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const uint32_t nb = gridDim.x;
  lds[threadIdx.x] = (char)threadIdx.x;  // touch the LDS allocation (residency is what matters)
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t e = 0; e < iters; ++e) {
    if (kStoreB) {
      uint4* my = box + (size_t)blockIdx.x * (kStoreB / 16);
      for (int i = threadIdx.x; i < kStoreB / 16; i += 64) my[i] = make_uint4(e, i, blockIdx.x, 0);
    }
    if (!asim::grid_barrier<kFence>(ctl, nb, e)) break;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <bool kFence, int kStoreB>
static double run(int nblocks, uint32_t iters, size_t lds, GpuCtl* ctl, uint4* box, uint64_t* cyc) {
  UB_CHECK(hipFuncSetAttribute((const void*)ub_barrier_kernel<kFence, kStoreB>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  UbTimer t;
  double best = 1e30;
  for (int r = 0; r < 5; ++r) {
    UB_CHECK(hipMemset(ctl, 0, sizeof(GpuCtl)));
    t.start();
    hipLaunchKernelGGL((ub_barrier_kernel<kFence, kStoreB>), dim3(nblocks), dim3(64), lds, 0, ctl, iters, box, cyc);
    best = std::min(best, t.stop_ms() * 1e3);
    UB_CHECK(hipDeviceSynchronize());
  }
  GpuCtl h;
  UB_CHECK(hipMemcpy(&h, ctl, sizeof(GpuCtl), hipMemcpyDeviceToHost));
  if (h.error) {
    printf("  barrier timed out (blocks not co-resident)\n");
    return -1;
  }
  return best / iters;
}

int main() {
  UbDevice dev;
  const int cus = dev.cus();
  printf("device %s, %d CUs\n", dev.p.gcnArchName, cus);
  GpuCtl* ctl;
  uint4* box;
  uint64_t* cyc;
  UB_CHECK(hipMalloc(&ctl, sizeof(GpuCtl)));
  UB_CHECK(hipMalloc(&box, (size_t)cus * 2048));
  UB_CHECK(hipMalloc(&cyc, sizeof(uint64_t) * cus));
  const uint32_t iters = 4000;
  const size_t lds = 128 * 1024;  // one block per CU, like the engine
  for (int nb : {8, 32, 112, 224, cus}) {
    if (nb > cus) continue;
    const double a = run<true, 0>(nb, iters, lds, ctl, box, cyc);
    const double b = run<false, 0>(nb, iters, lds, ctl, box, cyc);
    const double c = run<true, 2048>(nb, iters, lds, ctl, box, cyc);
    printf("grid barrier, %3d blocks: %.2f us (fenced), %.2f us (no fences), %.2f us (fenced, 2 KB stores/block)\n",
           nb, a, b, c);
  }
  return 0;
}
