// lud-shaped blocked LU decomposition (Rodinia lud: per 16-wide step, the
// diagonal tile is factorised by one block, the perimeter kernel solves the
// row and column tiles beside it, the internal kernel updates the trailing
// matrix with 16x16 tile products), plain HIP.  Usage: lud <dim, multiple of 16>
#include <cmath>

#include "app_common.h"

constexpr int BS = 16;

__global__ void lud_diagonal(float* m, int dim, int off) {
  __shared__ float sh[BS][BS];
  const int t = threadIdx.x;
  for (int i = 0; i < BS; ++i) sh[i][t] = m[(size_t)(off + i) * dim + off + t];
  __syncthreads();
  for (int i = 0; i < BS - 1; ++i) {
    if (t > i) {  // column i below the pivot (L), then row i+1.. of U
      for (int j = 0; j < i; ++j) sh[t][i] -= sh[t][j] * sh[j][i];
      sh[t][i] /= sh[i][i];
    }
    __syncthreads();
    if (t > i) {
      for (int j = 0; j < i + 1; ++j) sh[i + 1][t] -= sh[i + 1][j] * sh[j][t];
    }
    __syncthreads();
  }
  for (int i = 1; i < BS; ++i) m[(size_t)(off + i) * dim + off + t] = sh[i][t];
}

// blocks: one per tile right of (row strip) and below (column strip) the diagonal
__global__ void lud_perimeter(float* m, int dim, int off) {
  __shared__ float dia[BS][BS], row[BS][BS], col[BS][BS];
  const int t = threadIdx.x, b = blockIdx.x;
  const int r0 = off, c0 = off + (b + 1) * BS;  // row-strip tile
  for (int i = 0; i < BS; ++i) {
    dia[i][t] = m[(size_t)(off + i) * dim + off + t];
    row[i][t] = m[(size_t)(r0 + i) * dim + c0 + t];
    col[i][t] = m[(size_t)(c0 + i) * dim + off + t];
  }
  __syncthreads();
  // U of the row strip: forward substitution with unit-lower L (column t)
  for (int i = 1; i < BS; ++i)
    for (int j = 0; j < i; ++j) row[i][t] -= dia[i][j] * row[j][t];
  // L of the column strip: row t solves against U of the diagonal
  for (int i = 0; i < BS; ++i) {
    for (int j = 0; j < i; ++j) col[t][i] -= col[t][j] * dia[j][i];
    col[t][i] /= dia[i][i];
  }
  __syncthreads();
  for (int i = 0; i < BS; ++i) {
    m[(size_t)(r0 + i) * dim + c0 + t] = row[i][t];
    m[(size_t)(c0 + i) * dim + off + t] = col[i][t];
  }
}

__global__ void lud_internal(float* m, int dim, int off) {
  __shared__ float l[BS][BS], u[BS][BS];
  const int tx = threadIdx.x, ty = threadIdx.y;
  const int gr = off + (blockIdx.y + 1) * BS + ty, gc = off + (blockIdx.x + 1) * BS + tx;
  l[ty][tx] = m[(size_t)gr * dim + off + tx];
  u[ty][tx] = m[(size_t)(off + ty) * dim + gc];
  __syncthreads();
  float s = 0.f;
  for (int k = 0; k < BS; ++k) s += l[ty][k] * u[k][tx];
  m[(size_t)gr * dim + gc] -= s;
}

int main(int argc, char** argv) {
  const int dim = argc > 1 ? atoi(argv[1]) : 1024;
  std::vector<float> a((size_t)dim * dim);
  uint32_t s = 5;
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) {
      s = s * 1664525u + 1013904223u;
      a[(size_t)i * dim + j] = (float)(s >> 8) / 16777216.f + (i == j ? (float)dim : 0.f);  // diagonally dominant
    }
  float* d;
  APP_HIP(hipMalloc(&d, a.size() * 4));
  APP_HIP(hipMemcpy(d, a.data(), a.size() * 4, hipMemcpyHostToDevice));
  int off = 0;
  for (; off < dim - BS; off += BS) {
    lud_diagonal<<<1, BS>>>(d, dim, off);
    const int n = (dim - off) / BS - 1;
    lud_perimeter<<<n, BS>>>(d, dim, off);
    lud_internal<<<dim3(n, n), dim3(BS, BS)>>>(d, dim, off);
  }
  lud_diagonal<<<1, BS>>>(d, dim, off);
  APP_HIP(hipGetLastError());
  std::vector<float> lu(a.size());
  APP_HIP(hipMemcpy(lu.data(), d, lu.size() * 4, hipMemcpyDeviceToHost));
  // check rows of L*U against A
  double err = 0;
  for (int i = 0; i < dim; i += std::max(1, dim / 17))
    for (int j = 0; j < dim; ++j) {
      double v = 0;
      for (int k = 0; k <= std::min(i, j); ++k) v += (k == i ? 1.0 : lu[(size_t)i * dim + k]) * lu[(size_t)k * dim + j];
      err = std::max(err, std::fabs(v - a[(size_t)i * dim + j]) / (double)dim);
    }
  const bool ok = err < 1e-4;
  printf("lud dim=%d: max rel err %.2e %s\n", dim, err, ok ? "PASSED" : "FAILED");
  APP_HIP(hipFree(d));
  return ok ? 0 : 1;
}
