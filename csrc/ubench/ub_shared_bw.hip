// LDS bandwidth per CU (reference GPU_Microbenchmark shd/shared_bw,
// shared_bw_64, shared_lat).  16 waves per CU read LDS with conflict-free
// lane-linear addresses at 4, 8 and 16 bytes per lane (ds_read_b32 / _b64 /
// _b128), 8 independent reads in flight per lane; bytes per shader cycle per
// CU from the in-kernel clock of workgroup 0 (every CU runs the same work).
// The model's LDS path (shared-memory latency and bank-conflict degree per
// instruction) takes -gpgpu_smem_latency and -gpgpu_shmem_num_banks from
// ub_lds; this program records the width-dependent throughput for the
// correlation notes.
#include "ubench.h"

template <int W>
struct Vec;
template <>
struct Vec<4> { using T = uint32_t; };
template <>
struct Vec<8> { using T = uint2; };
template <>
struct Vec<16> { using T = uint4; };

__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int W>
__global__ void __launch_bounds__(1024) lds_bw(int iters, uint64_t* out, uint32_t* sink) {
  using T = typename Vec<W>::T;
  __shared__ T buf[1024 * 8];
  const int tid = threadIdx.x;
  for (int i = tid; i < 1024 * 8; i += blockDim.x) {
    T v;
    memset(&v, 0, sizeof(v));
    *reinterpret_cast<uint32_t*>(&v) = (uint32_t)i;
    buf[i] = v;
  }
  __syncthreads();
  uint32_t acc = 0;
  int base = tid & 1023;
  const uint64_t t0 = ub_clock();
  for (int it = 0; it < iters; ++it) {
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = buf[(base + k * 1024) & (1024 * 8 - 1)];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += fold(v[k]);
    base = (base + (int)(acc & 1u)) & 1023;  // keeps the loads live, stays lane-linear
  }
  __syncthreads();
  const uint64_t t1 = ub_clock();
  if (tid == 0 && blockIdx.x == 0) out[0] = t1 - t0;
  if (acc == 0xdeadbeefu) sink[0] = acc;
}

template <int W>
static double run(int cus, uint64_t* o, uint32_t* sink) {
  const int iters = 2048, threads = 1024;
  hipLaunchKernelGGL((lds_bw<W>), dim3(cus), dim3(threads), 0, 0, 16, o, sink);
  hipLaunchKernelGGL((lds_bw<W>), dim3(cus), dim3(threads), 0, 0, iters, o, sink);
  UB_CHECK(hipDeviceSynchronize());
  uint64_t cyc = 0;
  UB_CHECK(hipMemcpy(&cyc, o, 8, hipMemcpyDeviceToHost));
  const double bytes = (double)iters * 8 * threads * W;
  const double bpc = bytes / (double)cyc;
  printf("ds_read %2d B/lane: %7.1f bytes per cycle per CU\n", W, bpc);
  return bpc;
}

int main() {
  UbDevice dev;
  printf("device %s, %d CUs\n", dev.p.gcnArchName, dev.cus());
  uint64_t* o;
  uint32_t* sink;
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMalloc(&sink, 16));
  const double b4 = run<4>(dev.cus(), o, sink), b8 = run<8>(dev.cus(), o, sink), b16 = run<16>(dev.cus(), o, sink);
  printf("# lds_bytes_per_clk_per_cu_b32 %.1f\n# lds_bytes_per_clk_per_cu_b64 %.1f\n# lds_bytes_per_clk_per_cu_b128 %.1f\n",
         b4, b8, b16);
  // cycles one wave64 LDS read occupies the CU's LDS pipe (b32)
  printf("# lds_cycles_per_wave_read_b32 %.2f\n", 256.0 / b4);
  UB_CHECK(hipFree(o));
  UB_CHECK(hipFree(sink));
  return 0;
}
