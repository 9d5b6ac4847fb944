// Device functions called from a kernel and __constant__ / __device__ variables:
// the PC-relative (s_getpc_b64) and call patterns of tests/test_isatrace_binary.py
#include <hip/hip_runtime.h>
__device__ __noinline__ float f1(float x, const float* t) { return x * t[threadIdx.x & 7] + 1.0f; }
__device__ __noinline__ float f2(float x) { return sqrtf(x) * 3.0f; }
__constant__ float ctab[16] = {1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16};
__device__ float gvar[64];
__global__ void kcall(float* out, const float* t, int sel) {
  float x = out[threadIdx.x];
  x = sel ? f1(x, t) : f2(x);
  x += ctab[threadIdx.x & 15] + gvar[threadIdx.x & 63];
  out[threadIdx.x] = x;
}

