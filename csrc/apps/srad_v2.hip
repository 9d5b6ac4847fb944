// srad_v2-shaped speckle-reducing anisotropic diffusion (Rodinia srad_v2: per
// iteration the host derives q0^2 from the region-of-interest statistics of
// the image, kernel 1 computes the four directional derivatives and the
// diffusion coefficient of every pixel on 16x16 shared-memory tiles, kernel 2
// applies the divergence update), plain HIP.
// Usage: srad_v2 <rows> <cols> <lambda> <iterations>
#include <cmath>

#include "app_common.h"

constexpr int BS = 16;

__global__ void srad_cuda_1(float* dN, float* dS, float* dW, float* dE, float* c, const float* J, int rows, int cols,
                            float q0sqr) {
  __shared__ float t[BS + 2][BS + 2];
  const int tx = threadIdx.x, ty = threadIdx.y;
  const int x = blockIdx.x * BS + tx, y = blockIdx.y * BS + ty;
  const int k = y * cols + x;
  t[ty + 1][tx + 1] = J[k];
  if (ty == 0) t[0][tx + 1] = J[(y > 0 ? y - 1 : 0) * cols + x];
  if (ty == BS - 1) t[BS + 1][tx + 1] = J[(y + 1 < rows ? y + 1 : rows - 1) * cols + x];
  if (tx == 0) t[ty + 1][0] = J[y * cols + (x > 0 ? x - 1 : 0)];
  if (tx == BS - 1) t[ty + 1][BS + 1] = J[y * cols + (x + 1 < cols ? x + 1 : cols - 1)];
  __syncthreads();
  const float jc = t[ty + 1][tx + 1];
  const float n = t[ty][tx + 1] - jc, s = t[ty + 2][tx + 1] - jc, w = t[ty + 1][tx] - jc, e = t[ty + 1][tx + 2] - jc;
  const float g2 = (n * n + s * s + w * w + e * e) / (jc * jc);
  const float l = (n + s + w + e) / jc;
  const float num = 0.5f * g2 - (1.0f / 16.0f) * (l * l);
  float den = 1.f + 0.25f * l;
  const float qsqr = num / (den * den);
  den = (qsqr - q0sqr) / (q0sqr * (1.f + q0sqr));
  float cc = 1.f / (1.f + den);
  cc = cc < 0.f ? 0.f : (cc > 1.f ? 1.f : cc);
  dN[k] = n;
  dS[k] = s;
  dW[k] = w;
  dE[k] = e;
  c[k] = cc;
}

__global__ void srad_cuda_2(const float* dN, const float* dS, const float* dW, const float* dE, const float* c,
                            float* J, int rows, int cols, float lambda) {
  __shared__ float cs[BS + 1][BS + 1];
  const int tx = threadIdx.x, ty = threadIdx.y;
  const int x = blockIdx.x * BS + tx, y = blockIdx.y * BS + ty;
  const int k = y * cols + x;
  cs[ty][tx] = c[k];
  if (ty == BS - 1) cs[BS][tx] = c[(y + 1 < rows ? y + 1 : rows - 1) * cols + x];
  if (tx == BS - 1) cs[ty][BS] = c[y * cols + (x + 1 < cols ? x + 1 : cols - 1)];
  __syncthreads();
  const float cn = cs[ty][tx], cs_ = cs[ty + 1][tx], cw = cs[ty][tx], ce = cs[ty][tx + 1];
  const float d = cn * dN[k] + cs_ * dS[k] + cw * dW[k] + ce * dE[k];
  J[k] = J[k] + 0.25f * lambda * d;
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 1024, cols = argc > 2 ? atoi(argv[2]) : rows;
  const float lambda = argc > 3 ? (float)atof(argv[3]) : 0.5f;
  const int iters = argc > 4 ? atoi(argv[4]) : 2;
  const size_t n = (size_t)rows * cols;
  std::vector<float> J(n);
  for (size_t i = 0; i < n; ++i) J[i] = std::exp(0.5f + 0.4f * std::sin(0.013f * (float)i) * std::cos(0.007f * (float)i));
  float *dJ, *dN, *dS, *dW, *dE, *dc;
  for (float** p : {&dJ, &dN, &dS, &dW, &dE, &dc}) APP_HIP(hipMalloc(p, n * 4));
  APP_HIP(hipMemcpy(dJ, J.data(), n * 4, hipMemcpyHostToDevice));
  const dim3 grid(cols / BS, rows / BS), blk(BS, BS);
  for (int it = 0; it < iters; ++it) {
    double sum = 0, sum2 = 0;  // region of interest = whole image
    for (size_t i = 0; i < n; ++i) {
      sum += J[i];
      sum2 += (double)J[i] * J[i];
    }
    const double mean = sum / n, var = sum2 / n - mean * mean;
    const float q0sqr = (float)(var / (mean * mean));
    srad_cuda_1<<<grid, blk>>>(dN, dS, dW, dE, dc, dJ, rows, cols, q0sqr);
    srad_cuda_2<<<grid, blk>>>(dN, dS, dW, dE, dc, dJ, rows, cols, lambda);
    APP_HIP(hipGetLastError());
    APP_HIP(hipMemcpy(J.data(), dJ, n * 4, hipMemcpyDeviceToHost));
  }
  double s = 0;
  bool finite = true;
  for (size_t i = 0; i < n; ++i) {
    s += J[i];
    finite = finite && std::isfinite(J[i]);
  }
  const bool ok = finite && s / n > 0.5 && s / n < 5.0;
  printf("srad_v2 %dx%d iters=%d: mean %.5f %s\n", rows, cols, iters, s / n, ok ? "PASSED" : "FAILED");
  for (float* p : {dJ, dN, dS, dW, dE, dc}) APP_HIP(hipFree(p));
  return ok ? 0 : 1;
}
