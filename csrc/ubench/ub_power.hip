// UB_LIBS: -lamd_smi -lpthread
// Power validation micro-benchmarks (reference util/accelwattch
// accelwattch_hw_profiler/measureGpuPower.cpp + the AccelWattch ubench set):
// each stress kernel runs back to back for ~2 s while a host thread samples
// socket power through amd-smi every 10 ms; prints a CSV in the layout of
// hw_power_validation_*.csv (",mean HW_power,st_dev,var,#samples").
#include <amd_smi/amdsmi.h>

#include <atomic>
#include <functional>
#include <chrono>
#include <cmath>
#include <thread>

#include "ubench.h"

__global__ void k_idle() {}

__global__ void k_fp32(float* sink, int iters) {
  float x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x + k;
  for (int i = 0; i < iters; ++i)
    for (int k = 0; k < 8; ++k) x[k] = __builtin_fmaf(x[k], 1.000001f, 0.25f);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += x[k];
  if (s == -1.f) sink[0] = s;
}

__global__ void k_int(float* sink, int iters) {
  unsigned x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 7 + k;
  for (int i = 0; i < iters; ++i)
    for (int k = 0; k < 8; ++k) x[k] = x[k] * 1664525u + 1013904223u;
  unsigned s = 0;
  for (int k = 0; k < 8; ++k) s ^= x[k];
  if (s == 7u) sink[0] = (float)s;
}

__global__ void k_fp64(float* sink, int iters) {
  double x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x + k;
  for (int i = 0; i < iters; ++i)
    for (int k = 0; k < 8; ++k) x[k] = __builtin_fma(x[k], 1.000001, 0.25);
  double s = 0;
  for (int k = 0; k < 8; ++k) s += x[k];
  if (s == -1.0) sink[0] = (float)s;
}

__global__ void k_sfu(float* sink, int iters) {
  float x = threadIdx.x + 1.5f;
  for (int i = 0; i < iters; ++i) x = __builtin_sqrtf(x) + __expf(-x) + 1.0f;
  if (x == -1.f) sink[0] = x;
}

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;

__global__ void k_mfma(float* sink, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)0.5f;
  }
  f32x16 c0 = {}, c1 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  if (s == -1.f) sink[0] = s;
}

__global__ void k_lds(float* sink, int iters) {
  __shared__ float s[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) s[i] = (float)i;
  __syncthreads();
  float acc = 0;
  unsigned idx = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    acc += s[idx & 4095];
    idx += 64;
  }
  if (acc == -1.f) sink[0] = acc;
}

__global__ void k_hbm(const float4* __restrict__ a, size_t n, float* sink) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    acc.x += v.x;
    acc.w += v.w;
  }
  if (acc.x + acc.w == 1234.5f) sink[0] = acc.x;
}

struct Sampler {
  amdsmi_processor_handle h = nullptr;
  bool ok = false;
  Sampler(int hip_dev) {
    if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return;
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), hip_dev) != hipSuccess) return;
    unsigned dom = 0, b = 0, dv = 0, fn = 0;
    sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn);
    uint32_t ns = 0;
    amdsmi_get_socket_handles(&ns, nullptr);
    std::vector<amdsmi_socket_handle> socks(ns);
    amdsmi_get_socket_handles(&ns, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      amdsmi_get_processor_handles(s, &np, nullptr);
      std::vector<amdsmi_processor_handle> ps(np);
      amdsmi_get_processor_handles(s, &np, ps.data());
      for (auto p : ps) {
        amdsmi_bdf_t bdf;
        if (amdsmi_get_gpu_device_bdf(p, &bdf) != AMDSMI_STATUS_SUCCESS) continue;
        if (bdf.bus_number == b && bdf.device_number == dv && bdf.function_number == fn) {
          h = p;
          ok = true;
        }
      }
    }
  }
  double watts() const {
    amdsmi_power_info_t pi;
    if (!ok || amdsmi_get_power_info(h, &pi) != AMDSMI_STATUS_SUCCESS) return NAN;
    if (pi.current_socket_power != UINT32_MAX && pi.current_socket_power) return pi.current_socket_power;
    if (pi.average_socket_power != UINT32_MAX && pi.average_socket_power) return pi.average_socket_power;
    return (double)pi.socket_power;
  }
  ~Sampler() {
    if (ok) amdsmi_shut_down();
  }
};

int main(int argc, char** argv) {
  UbDevice d;
  Sampler smi(d.dev);
  if (!smi.ok) {
    printf("# amd-smi power sampling unavailable on this node; nothing measured\n");
    return 0;
  }
  const double secs = argc > 1 ? atof(argv[1]) : 2.0;
  const int cus = d.cus();
  float* sink;
  UB_CHECK(hipMalloc(&sink, 64));
  const size_t hbm_bytes = (size_t)1 << 30;
  float4* buf;
  UB_CHECK(hipMalloc(&buf, hbm_bytes));
  UB_CHECK(hipMemset(buf, 0, hbm_bytes));
  struct K {
    const char* name;
    std::function<void()> launch;
  };
  const dim3 g(cus * 8), b(256);
  std::vector<K> ks = {
      {"idle", [&] { hipLaunchKernelGGL(k_idle, dim3(1), dim3(64), 0, 0); }},
      {"fp32_fma", [&] { hipLaunchKernelGGL(k_fp32, g, b, 0, 0, sink, 20000); }},
      {"int32_mad", [&] { hipLaunchKernelGGL(k_int, g, b, 0, 0, sink, 20000); }},
      {"fp64_fma", [&] { hipLaunchKernelGGL(k_fp64, g, b, 0, 0, sink, 10000); }},
      {"sfu_sqrt_exp", [&] { hipLaunchKernelGGL(k_sfu, g, b, 0, 0, sink, 20000); }},
      {"mfma_bf16", [&] { hipLaunchKernelGGL(k_mfma, g, b, 0, 0, sink, 4000); }},
      {"lds_read", [&] { hipLaunchKernelGGL(k_lds, g, b, 0, 0, sink, 20000); }},
      {"hbm_read", [&] { hipLaunchKernelGGL(k_hbm, dim3(4096), b, 0, 0, buf, hbm_bytes / 16, sink); }},
  };
  printf(",mean HW_power,st_dev,var,#samples\n");
  for (auto& k : ks) {
    k.launch();
    UB_CHECK(hipDeviceSynchronize());
    std::atomic<bool> stop{false};
    std::vector<double> samples;
    std::thread th([&] {
      while (!stop.load()) {
        double w = smi.watts();
        if (!std::isnan(w)) samples.push_back(w);
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    });
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
      for (int r = 0; r < 4; ++r) k.launch();
      UB_CHECK(hipDeviceSynchronize());
    }
    stop = true;
    th.join();
    // drop the first quarter (ramp-up), like the reference's steady window
    const size_t skip = samples.size() / 4;
    double m = 0, v = 0;
    const size_t n = samples.size() - skip;
    for (size_t i = skip; i < samples.size(); ++i) m += samples[i];
    m = n ? m / n : NAN;
    for (size_t i = skip; i < samples.size(); ++i) v += (samples[i] - m) * (samples[i] - m);
    v = n > 1 ? v / (n - 1) : 0;
    printf("%s,%.4f,%.4f,%.4f,%zu\n", k.name, m, std::sqrt(v), v, n);
    fflush(stdout);
  }
  UB_CHECK(hipFree(buf));
  UB_CHECK(hipFree(sink));
  return 0;
}
