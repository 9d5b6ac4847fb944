// Cache and LDS bandwidth by access width (reference GPU_Microbenchmark
// l1_cache/l1_bw_{32f,64f,128}, l2_cache/l2_bw_{32f,64f,128} and
// shd/shared_bw): every CU's workgroups re-read a working set that lives in
// the vector L1 (16 KB per workgroup), in the L2 (2 MB shared) or in LDS, with
// 4-, 8- and 16-byte loads per lane; bytes per cycle per CU.
#include "ubench.h"

template <class T>
__global__ void k_glob(const T* __restrict__ a, size_t mask, int reps, float* sink) {
  float acc = 0;
  const size_t base = (size_t)blockIdx.x * 0;  // every workgroup sweeps the same set
  for (int r = 0; r < reps; ++r)
    for (size_t i = threadIdx.x; i <= mask; i += blockDim.x) {
      const T v = a[(base + i + (size_t)r * 64) & mask];
      acc += reinterpret_cast<const float*>(&v)[0];
    }
  if (acc == -1.f) sink[0] = acc;
}

template <class T>
__global__ void k_lds(int reps, float* sink) {
  __shared__ T s[2048];
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) reinterpret_cast<float*>(&s[i])[0] = (float)i;
  __syncthreads();
  float acc = 0;
  for (int r = 0; r < reps; ++r) {
    const T v = s[(threadIdx.x + r * 64) & 2047];
    acc += reinterpret_cast<const float*>(&v)[0];
  }
  if (acc == -1.f) sink[0] = acc;
}

template <class T>
static double glob_bw(const void* buf, size_t bytes, int cus, double mhz, float* sink) {
  const size_t n = bytes / sizeof(T);
  const int reps = 64, blocks = cus * 4;
  UbTimer t;
  hipLaunchKernelGGL(k_glob<T>, dim3(blocks), dim3(256), 0, 0, (const T*)buf, n - 1, 2, sink);  // warm
  t.start();
  hipLaunchKernelGGL(k_glob<T>, dim3(blocks), dim3(256), 0, 0, (const T*)buf, n - 1, reps, sink);
  const double ms = t.stop_ms();
  const double moved = (double)blocks * reps * n * sizeof(T);
  return moved / (ms * 1e-3 * mhz * 1e6) / cus;
}

template <class T>
static double lds_bw(int cus, double mhz, float* sink) {
  const int reps = 1 << 14, blocks = cus * 4;
  UbTimer t;
  t.start();
  hipLaunchKernelGGL(k_lds<T>, dim3(blocks), dim3(256), 0, 0, reps, sink);
  const double ms = t.stop_ms();
  return (double)blocks * 256 * reps * sizeof(T) / (ms * 1e-3 * mhz * 1e6) / cus;
}

int main() {
  UbDevice d;
  const double mhz = ub_shader_mhz();
  const int cus = d.cus();
  float* sink;
  void* buf;
  UB_CHECK(hipMalloc(&sink, 16));
  UB_CHECK(hipMalloc(&buf, 2 << 20));
  UB_CHECK(hipMemset(buf, 0, 2 << 20));
  printf("# measured_shader_mhz %.1f\n", mhz);
  const size_t l1 = 16 << 10, l2 = 2 << 20;
  printf("l1_bw  32b %7.1f  64b %7.1f  128b %7.1f B/clk/CU\n", glob_bw<float>(buf, l1, cus, mhz, sink),
         glob_bw<float2>(buf, l1, cus, mhz, sink), glob_bw<float4>(buf, l1, cus, mhz, sink));
  printf("l2_bw  32b %7.1f  64b %7.1f  128b %7.1f B/clk/CU\n", glob_bw<float>(buf, l2, cus, mhz, sink),
         glob_bw<float2>(buf, l2, cus, mhz, sink), glob_bw<float4>(buf, l2, cus, mhz, sink));
  printf("lds_bw 32b %7.1f  64b %7.1f  128b %7.1f B/clk/CU\n", lds_bw<float>(cus, mhz, sink),
         lds_bw<float2>(cus, mhz, sink), lds_bw<float4>(cus, mhz, sink));
  UB_CHECK(hipFree(sink));
  UB_CHECK(hipFree(buf));
  return 0;
}
