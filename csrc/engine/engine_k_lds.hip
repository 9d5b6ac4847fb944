// engine_kernel instantiations: the LDS-state builds (one unit resident per block, or time-sliced).
// Separate translation units so the builds compile in parallel.
#include "engine_kernel.h"

namespace asim {

template __global__ void engine_kernel<WavePar, false, kModeLds>(GpuArgs);
template __global__ void engine_kernel<WavePar, true, kModeLds>(GpuArgs);

ASIM_ENGINE_CFG_UPLOAD(lds)

}  // namespace asim
