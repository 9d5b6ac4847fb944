// backprop-shaped neural-network training step (Rodinia backprop: one input
// layer of N units, 16 hidden units, one output; the layer-forward kernel
// multiplies 16x16 weight tiles by the input slice and reduces the columns in
// shared memory, the adjust-weights kernel applies the momentum update),
// plain HIP.  Usage: backprop <input units, multiple of 16>
#include <cmath>

#include "app_common.h"

constexpr int BS = 16;
constexpr float kEta = 0.3f, kMom = 0.3f;

__global__ void bpnn_layerforward(const float* input, float* w, float* partial, int hid) {
  __shared__ float in_node[BS];
  __shared__ float wm[BS][BS];
  const int by = blockIdx.y, tx = threadIdx.x, ty = threadIdx.y;
  const int idx = (hid + 1) * BS * by + (hid + 1) * ty + tx + 1 + (hid + 1);
  if (tx == 0) in_node[ty] = input[BS * by + ty + 1];
  __syncthreads();
  wm[ty][tx] = w[idx] * in_node[ty];
  __syncthreads();
  for (int p = 2; p <= BS; p *= 2) {  // column sums by halving strides
    if (ty % p == 0) wm[ty][tx] += wm[ty + p / 2][tx];
    __syncthreads();
  }
  w[idx] = wm[ty][tx];
  __syncthreads();
  if (tx == 0) partial[by * hid + ty] = wm[0][ty];
}

__global__ void bpnn_adjust_weights(const float* delta, int hid, const float* ly, float* w, float* oldw) {
  const int by = blockIdx.y, tx = threadIdx.x, ty = threadIdx.y;
  const int idx = (hid + 1) * BS * by + (hid + 1) * ty + tx + 1 + (hid + 1);
  const int iy = BS * by + ty + 1, ix = tx + 1;
  const float d = kEta * delta[ix] * ly[iy] + kMom * oldw[idx];
  w[idx] += d;
  oldw[idx] = d;
  __syncthreads();
  if (ty == 0 && by == 0) {
    const float b = kEta * delta[ix] + kMom * oldw[ix];
    w[ix] += b;
    oldw[ix] = b;
  }
}

int main(int argc, char** argv) {
  const int in = argc > 1 ? atoi(argv[1]) : 65536, hid = BS, blocks = in / BS;
  const size_t nw = (size_t)(in + 1) * (hid + 1);
  std::vector<float> input(in + 1), w(nw), oldw(nw, 0.f), delta(hid + 1);
  uint32_t s = 9;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)(s >> 8) / 16777216.f; };
  for (auto& v : input) v = rnd();
  for (auto& v : w) v = rnd() - 0.5f;
  for (auto& v : delta) v = rnd() - 0.5f;
  float *d_in, *d_w, *d_old, *d_part, *d_delta;
  APP_HIP(hipMalloc(&d_in, input.size() * 4));
  APP_HIP(hipMalloc(&d_w, nw * 4));
  APP_HIP(hipMalloc(&d_old, nw * 4));
  APP_HIP(hipMalloc(&d_part, (size_t)blocks * hid * 4));
  APP_HIP(hipMalloc(&d_delta, delta.size() * 4));
  APP_HIP(hipMemcpy(d_in, input.data(), input.size() * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_w, w.data(), nw * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_old, oldw.data(), nw * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_delta, delta.data(), delta.size() * 4, hipMemcpyHostToDevice));
  const dim3 grid(1, blocks), blk(BS, BS);
  bpnn_layerforward<<<grid, blk>>>(d_in, d_w, d_part, hid);
  APP_HIP(hipGetLastError());
  std::vector<float> part((size_t)blocks * hid);
  APP_HIP(hipMemcpy(part.data(), d_part, part.size() * 4, hipMemcpyDeviceToHost));
  // hidden layer sums on the host (as the reference does), checked against a CPU forward pass
  bool ok = true;
  for (int j = 0; j < hid && ok; ++j) {
    double g = 0, r = 0;
    for (int b = 0; b < blocks; ++b) g += part[(size_t)b * hid + j];
    for (int k = 1; k <= in; ++k) r += (double)w[(size_t)k * (hid + 1) + j + 1] * input[k];
    ok = std::fabs(g - r) <= 1e-3 * (1.0 + std::fabs(r));
  }
  bpnn_adjust_weights<<<grid, blk>>>(d_delta, hid, d_in, d_w, d_old);
  APP_HIP(hipGetLastError());
  APP_HIP(hipDeviceSynchronize());
  std::vector<float> o2(nw);
  APP_HIP(hipMemcpy(o2.data(), d_old, nw * 4, hipMemcpyDeviceToHost));
  const size_t k = (size_t)(hid + 1) * 5 + 3;  // row 5, column 3
  ok = ok && std::fabs(o2[k] - kEta * delta[3] * input[5]) < 1e-5f;
  printf("backprop in=%d: %s\n", in, ok ? "PASSED" : "FAILED");
  for (float* p : {d_in, d_w, d_old, d_part, d_delta}) APP_HIP(hipFree(p));
  return ok ? 0 : 1;
}
