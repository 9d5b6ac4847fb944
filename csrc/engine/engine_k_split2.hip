// The split-state build compiled for two engine waves per SIMD: the hot
// prefix of an SM (~16 KB, sm.h) lets eight blocks share a CU's LDS, and
// amdgpu_waves_per_eu(2, 2) keeps the kernel within 256 vector + accumulation
// registers (the one-wave build uses ~420), so two waves share each SIMD and
// hide each other's LDS / L2 latency.  Selected with ASIM_GPU_SPLIT_WAVES=2
// (gpu_engine.hip split_waves()).
#include "engine_kernel.h"

namespace asim {

#define ASIM_SPLIT2_KERNEL_ATTRS __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))

__global__ void ASIM_SPLIT2_KERNEL_ATTRS engine_split2_kernel(GpuArgs a) {
  engine_body<WavePar, true, kModeSplit>(a, blockIdx.x);
}

ASIM_ENGINE_CFG_UPLOAD(split2)

}  // namespace asim
