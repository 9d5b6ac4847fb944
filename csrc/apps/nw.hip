// nw-shaped Needleman-Wunsch alignment (Rodinia nw: the (n+1)^2 score matrix
// is filled in 16x16 tiles along anti-diagonals; kernel 1 sweeps the upper-left
// triangle of tiles, kernel 2 the lower-right one; inside a tile the 16 threads
// walk the tile's anti-diagonals through shared memory), plain HIP.
// Usage: nw <sequence length, multiple of 16> <gap penalty>
#include <algorithm>
#include <cmath>

#include "app_common.h"

constexpr int BS = 16;

__device__ __forceinline__ int max3(int a, int b, int c) { return max(a, max(b, c)); }

// fill tile (bx, by) of the matrix: score[(by*BS + i) * cols + bx*BS + j]
__device__ __forceinline__ void nw_tile(const int* ref, int* score, int cols, int penalty, int bx, int by) {
  __shared__ int tmp[BS + 1][BS + 1];
  __shared__ int rf[BS][BS];
  const int tx = threadIdx.x;
  const int base = cols * BS * by + BS * bx;  // top-left corner (row/column 0 of the tile's halo)
  for (int ty = 0; ty < BS; ++ty) rf[ty][tx] = ref[base + cols * (ty + 1) + tx + 1];
  if (tx == 0) tmp[0][0] = score[base];
  tmp[tx + 1][0] = score[base + cols * (tx + 1)];
  tmp[0][tx + 1] = score[base + tx + 1];
  __syncthreads();
  for (int m = 0; m < BS; ++m) {  // upper-left half of the tile's anti-diagonals
    if (tx <= m) {
      const int x = tx + 1, y = m - tx + 1;
      tmp[y][x] = max3(tmp[y - 1][x - 1] + rf[y - 1][x - 1], tmp[y][x - 1] - penalty, tmp[y - 1][x] - penalty);
    }
    __syncthreads();
  }
  for (int m = BS - 2; m >= 0; --m) {  // lower-right half
    if (tx <= m) {
      const int x = tx + BS - m, y = BS - tx;
      tmp[y][x] = max3(tmp[y - 1][x - 1] + rf[y - 1][x - 1], tmp[y][x - 1] - penalty, tmp[y - 1][x] - penalty);
    }
    __syncthreads();
  }
  for (int ty = 0; ty < BS; ++ty) score[base + cols * (ty + 1) + tx + 1] = tmp[ty + 1][tx + 1];
}

__global__ void needle_cuda_shared_1(const int* ref, int* score, int cols, int penalty, int i) {
  nw_tile(ref, score, cols, penalty, blockIdx.x, i - 1 - blockIdx.x);
}

__global__ void needle_cuda_shared_2(const int* ref, int* score, int cols, int penalty, int i, int bw) {
  nw_tile(ref, score, cols, penalty, blockIdx.x + bw - i, bw - 1 - blockIdx.x);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2048, penalty = argc > 2 ? atoi(argv[2]) : 10;
  const int cols = n + 1, bw = n / BS;
  std::vector<int> s1(cols), s2(cols), ref((size_t)cols * cols), score((size_t)cols * cols, 0);
  uint32_t s = 7;
  for (int i = 1; i < cols; ++i) {
    s = s * 1664525u + 1013904223u;
    s1[i] = (int)((s >> 16) % 10) + 1;
    s = s * 1664525u + 1013904223u;
    s2[i] = (int)((s >> 16) % 10) + 1;
  }
  for (int i = 1; i < cols; ++i)
    for (int j = 1; j < cols; ++j) ref[(size_t)i * cols + j] = (s1[i] == s2[j]) ? 5 : -3 + (int)((i * 7 + j) % 3);
  for (int i = 1; i < cols; ++i) score[(size_t)i * cols] = -i * penalty;
  for (int j = 1; j < cols; ++j) score[j] = -j * penalty;
  int *d_ref, *d_score;
  APP_HIP(hipMalloc(&d_ref, ref.size() * 4));
  APP_HIP(hipMalloc(&d_score, score.size() * 4));
  APP_HIP(hipMemcpy(d_ref, ref.data(), ref.size() * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(d_score, score.data(), score.size() * 4, hipMemcpyHostToDevice));
  for (int i = 1; i <= bw; ++i) needle_cuda_shared_1<<<i, BS>>>(d_ref, d_score, cols, penalty, i);
  for (int i = bw - 1; i >= 1; --i) needle_cuda_shared_2<<<i, BS>>>(d_ref, d_score, cols, penalty, i, bw);
  APP_HIP(hipGetLastError());
  std::vector<int> out(score.size());
  APP_HIP(hipMemcpy(out.data(), d_score, out.size() * 4, hipMemcpyDeviceToHost));
  for (int i = 1; i < cols; ++i)
    for (int j = 1; j < cols; ++j) {
      const size_t k = (size_t)i * cols + j;
      score[k] = std::max({score[k - cols - 1] + ref[k], score[k - 1] - penalty, score[k - cols] - penalty});
    }
  const bool ok = out == score;
  printf("nw n=%d penalty=%d: %s\n", n, penalty, ok ? "PASSED" : "FAILED");
  APP_HIP(hipFree(d_ref));
  APP_HIP(hipFree(d_score));
  return ok ? 0 : 1;
}
