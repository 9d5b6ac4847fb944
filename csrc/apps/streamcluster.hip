// streamcluster-shaped online clustering (Rodinia streamcluster: the pgain
// step evaluates opening a candidate centre x -- every point computes its
// weighted distance to x in the d-dimensional coordinate array (stored
// dimension-major), marks whether it would switch and accumulates the cost
// change per current centre into per-thread work memory; the host sums the
// work memory and accepts or rejects the candidate), plain HIP.
// Usage: streamcluster <points> <dims> <candidates> <initial centres>
#include <cmath>

#include "app_common.h"

constexpr int kThreads = 512;

__global__ void kernel_compute_cost(int num, int dim, int x, const float* coord, const float* weight,
                                    const float* cost, const int* assign, const int* center_table, int K,
                                    float* work_mem, int* switch_membership) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= num) return;
  float* lower = work_mem + (size_t)tid * (K + 1);
  float d2 = 0.f;
  for (int i = 0; i < dim; ++i) {
    const float t = coord[(size_t)i * num + x] - coord[(size_t)i * num + tid];
    d2 += t * t;
  }
  const float x_cost = d2 * weight[tid];
  const float c = cost[tid];
  for (int k = 0; k <= K; ++k) lower[k] = 0.f;
  if (x_cost < c) {
    switch_membership[tid] = 1;
    lower[K] += x_cost - c;
  } else {
    lower[center_table[assign[tid]]] += c - x_cost;
  }
}

int main(int argc, char** argv) {
  const int num = argc > 1 ? atoi(argv[1]) : 65536, dim = argc > 2 ? atoi(argv[2]) : 16;
  const int cands = argc > 3 ? atoi(argv[3]) : 24, K = argc > 4 ? atoi(argv[4]) : 6;
  std::vector<float> coord((size_t)dim * num), weight(num, 1.f), cost(num);
  std::vector<int> assign(num), table(num, 0);
  uint32_t s = 11;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)(s >> 8) / 16777216.f; };
  for (auto& v : coord) v = rnd();
  for (int k = 0; k < K; ++k) table[k] = k;
  auto dist2 = [&](int a, int b) {
    float d = 0;
    for (int i = 0; i < dim; ++i) {
      const float t = coord[(size_t)i * num + a] - coord[(size_t)i * num + b];
      d += t * t;
    }
    return d;
  };
  for (int p = 0; p < num; ++p) {  // initial assignment to centres 0..K-1
    int best = 0;
    for (int k = 1; k < K; ++k)
      if (dist2(p, k) < dist2(p, best)) best = k;
    assign[p] = best;
    cost[p] = dist2(p, best) * weight[p];
  }
  float *d_coord, *d_w, *d_cost, *d_work;
  int *d_assign, *d_table, *d_switch;
  APP_HIP(hipMalloc(&d_coord, coord.size() * 4));
  APP_HIP(hipMalloc(&d_w, num * 4));
  APP_HIP(hipMalloc(&d_cost, num * 4));
  APP_HIP(hipMalloc(&d_work, (size_t)num * (K + 1) * 4));
  APP_HIP(hipMalloc(&d_assign, num * 4));
  APP_HIP(hipMalloc(&d_table, num * 4));
  APP_HIP(hipMalloc(&d_switch, num * 4));
  APP_HIP(hipMemcpy(d_coord, coord.data(), coord.size() * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_w, weight.data(), num * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_table, table.data(), num * 4, hipMemcpyHostToDevice));
  std::vector<float> work((size_t)num * (K + 1));
  std::vector<int> sw(num);
  bool ok = true;
  int opened = 0;
  for (int c = 0; c < cands; ++c) {
    const int x = (int)(rnd() * (num - 1));
    APP_HIP(hipMemcpy(d_cost, cost.data(), num * 4, hipMemcpyHostToDevice));
    APP_HIP(hipMemcpy(d_assign, assign.data(), num * 4, hipMemcpyHostToDevice));
    APP_HIP(hipMemset(d_switch, 0, num * 4));
    kernel_compute_cost<<<(num + kThreads - 1) / kThreads, kThreads>>>(num, dim, x, d_coord, d_w, d_cost, d_assign,
                                                                       d_table, K, d_work, d_switch);
    APP_HIP(hipGetLastError());
    APP_HIP(hipMemcpy(work.data(), d_work, work.size() * 4, hipMemcpyDeviceToHost));
    APP_HIP(hipMemcpy(sw.data(), d_switch, num * 4, hipMemcpyDeviceToHost));
    double gain = 0;  // accept the candidate if switching points lowers the total cost
    for (int p = 0; p < num; ++p) gain -= work[(size_t)p * (K + 1) + K];
    const int probe = c * 7919 % num;  // spot check one point against the host
    const float xc = dist2(probe, x) * weight[probe];
    ok = ok && (sw[probe] == (xc < cost[probe] ? 1 : 0));
    if (gain > 0 && K + opened < num) {
      for (int p = 0; p < num; ++p)
        if (sw[p]) {
          assign[p] = K - 1;  // re-use the last table slot for the opened centre
          cost[p] = dist2(p, x) * weight[p];
        }
      ++opened;
    }
  }
  printf("streamcluster n=%d d=%d candidates=%d opened=%d: %s\n", num, dim, cands, opened, ok ? "PASSED" : "FAILED");
  for (void* p : {(void*)d_coord, (void*)d_w, (void*)d_cost, (void*)d_work, (void*)d_assign, (void*)d_table,
                  (void*)d_switch})
    APP_HIP(hipFree(p));
  return ok ? 0 : 1;
}
