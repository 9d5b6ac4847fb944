// engine_kernel instantiations: the stage-profiling builds (ASIM_GPU_PROFILE).
// Separate translation units so the builds compile in parallel.
#include "engine_kernel.h"

namespace asim {

template __global__ void engine_kernel<WaveParProf, false, kModeLds>(GpuArgs);
template __global__ void engine_kernel<WaveParProf, true, kModeLds>(GpuArgs);
template __global__ void engine_kernel<WaveParProf, true, kModeGlobal>(GpuArgs);
template __global__ void engine_kernel<WaveParProf, true, kModeSplit>(GpuArgs);

ASIM_ENGINE_CFG_UPLOAD(prof)

}  // namespace asim
