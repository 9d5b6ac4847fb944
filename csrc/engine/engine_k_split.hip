// engine_kernel instantiation: the split-state build (an SM's hot prefix in
// LDS, its geometry-sized arrays and every channel in HBM: sm_split.h).
// Separate translation unit so the builds compile in parallel.
#include "engine_kernel.h"

namespace asim {

template __global__ void engine_kernel<WavePar, true, kModeSplit>(GpuArgs);

__global__ void ASIM_ENGINE_KERNEL_ATTRS engine_batch_split_kernel(const GpuArgs* __restrict__ jobs,
                                                                   const uint16_t* __restrict__ block_job) {
  const uint32_t j = block_job[blockIdx.x];
  const GpuArgs a = jobs[j];
  engine_body<WavePar, true, kModeSplit>(a, blockIdx.x - a.block0);
}

ASIM_ENGINE_CFG_UPLOAD(split)

}  // namespace asim
