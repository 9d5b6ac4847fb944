// engine_kernel instantiations: the global-state build (units simulated in place in HBM) and the batch kernel.
// Separate translation units so the builds compile in parallel.
#include "engine_kernel.h"

namespace asim {

template __global__ void engine_kernel<WavePar, true, kModeGlobal>(GpuArgs);

__global__ void ASIM_ENGINE_KERNEL_ATTRS engine_batch_kernel(const GpuArgs* __restrict__ jobs,
                                                             const uint16_t* __restrict__ block_job) {
  const uint32_t j = block_job[blockIdx.x];
  const GpuArgs a = jobs[j];
  engine_body<WavePar, true, kModeGlobal>(a, blockIdx.x - a.block0);
}

ASIM_ENGINE_CFG_UPLOAD(global)

}  // namespace asim
