// Shared host helpers of the HIP application suite (plain HIP: the traces
// come from the automatic ISA tracer, accel_sim_framework_distributed_amd/
// isatrace, so the kernels carry no annotations).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define APP_HIP(x)                                                                                   \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);        \
      exit(3);                                                                                       \
    }                                                                                                \
  } while (0)
