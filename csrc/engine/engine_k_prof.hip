// engine_kernel instantiations: the stage-profiling builds (ASIM_GPU_PROFILE).
// Separate translation units so the builds compile in parallel.
#include "engine_kernel.h"

namespace asim {

template __global__ void engine_kernel<WaveParProf, false, false>(GpuArgs);
template __global__ void engine_kernel<WaveParProf, true, false>(GpuArgs);
template __global__ void engine_kernel<WaveParProf, true, true>(GpuArgs);

ASIM_ENGINE_CFG_UPLOAD(prof)

}  // namespace asim
