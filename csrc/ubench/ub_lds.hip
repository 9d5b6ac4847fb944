// LDS latency, bandwidth and bank structure (reference GPU_Microbenchmark
// shd/shared_lat, shared_bw, shd_config and l1_cache/l1_banks): a dependent
// ds_read chain for latency, all-lane reads for bandwidth, and a stride
// sweep whose slowdown reveals the bank count (conflict degree doubles each
// time the stride doubles past the bank-width wrap).
#include "ubench.h"

__global__ void lds_lat_kernel(int iters, uint64_t* out) {
  __shared__ uint32_t s[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) s[i] = (uint32_t)((i + 33) & 1023);
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t j = 0;
  asm volatile("v_mov_b32 %0, %0" : "+v"(j));
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) j = s[j];
  uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = j;
}

// lane l chases a self-loop at word (l * stride) % N: one wave-wide ds_read
// per step whose addresses follow the stride; four independent chains per
// lane keep the LDS pipe busy, so time per step tracks the conflict degree
__global__ void lds_stride_kernel(int stride, int iters, uint64_t* out) {
  __shared__ uint32_t s[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) s[i] = (uint32_t)i;  // s[a] = a: self loops
  __syncthreads();
  uint32_t a0 = (threadIdx.x * (uint32_t)stride) & 16383u;
  uint32_t a1 = a0 ^ 1u, a2 = a0 ^ 2u, a3 = a0 ^ 3u;  // same bank pattern, different words
  uint64_t t0 = ub_clock();
  for (int i = 0; i < iters; ++i) {
    a0 = s[a0];
    a1 = s[a1];
    a2 = s[a2];
    a3 = s[a3];
  }
  uint64_t t1 = ub_clock();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = a0 + a1 + a2 + a3;
  }
}

int main() {
  UbDevice d;
  uint64_t* o;
  UB_CHECK(hipMalloc(&o, 16));
  uint64_t h[2];
  const int iters = 4096;
  hipLaunchKernelGGL(lds_lat_kernel, dim3(1), dim3(64), 0, 0, iters, o);
  UB_CHECK(hipMemcpy(h, o, 16, hipMemcpyDeviceToHost));
  const double lat = (double)h[0] / iters;
  printf("LDS dependent-read latency %.1f cycles\n", lat);
  double base = 0, prev = 0;
  int banks = 0;
  for (int stride = 1; stride <= 128; stride *= 2) {
    hipLaunchKernelGGL(lds_stride_kernel, dim3(1), dim3(64), 0, 0, stride, iters, o);
    UB_CHECK(hipMemcpy(h, o, 16, hipMemcpyDeviceToHost));
    const double c = (double)h[0] / (iters * 4.0);
    if (stride == 1) base = c;
    printf("stride %3d words: %.2f cycles/read (x%.2f)\n", stride, c, c / base);
    // the slowdown stops growing once a half-wave (32 lanes are serviced per
    // LDS cycle) lands in one bank: that first saturated stride s/2 means
    // s/2 * 2 = s banks
    if (stride > 1 && !banks && prev > 0 && c < prev * 1.15 && c / base > 2.0) banks = stride;
    prev = c;
  }
  if (banks) printf("# lds_banks %d\n", banks);
  ub_opt("-gpgpu_smem_latency", (long long)(lat + 0.5));
  ub_opt("-gpgpu_shmem_num_banks", banks ? banks : 64);
  UB_CHECK(hipFree(o));
  return 0;
}
