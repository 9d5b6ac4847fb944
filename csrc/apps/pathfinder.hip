// pathfinder-shaped dynamic programming (Rodinia pathfinder: minimum-cost
// path down a 2-D wall, one row per step, the previous row staged in shared
// memory with a one-column halo), HIP + asim_trace annotations.
#include <cmath>

#include "../tracer/asim_trace.h"

using namespace asim_trace;

constexpr int B = 256;

template <class TR>
__global__ void dynproc(TR tr, const int* wall_row, const int* src, int* dst, int cols) {
  __shared__ int prev[B + 2];
  auto w = tr.wave();
  const int x = blockIdx.x * B + threadIdx.x;
  ASIM_VALU(w, V_MAD_U32_U24, 1, 0);
  ASIM_VALU(w, V_CMP_GT_I32, 0, 1);
  int v = 0x3fffffff;
  if (x < cols) v = ASIM_LD(w, GLOBAL_LOAD_DWORD, src + x, 2, 1);
  ASIM_VALU(w, S_WAITCNT, 0, 0);
  ASIM_ST(w, DS_WRITE_B32, &prev[threadIdx.x + 1], v, 2, 3);
  if (threadIdx.x == 0) {
    int h = 0x3fffffff;
    if (x > 0) h = ASIM_LD(w, GLOBAL_LOAD_DWORD, src + x - 1, 4, 1);
    ASIM_ST(w, DS_WRITE_B32, &prev[0], h, 4, 3);
  }
  if (threadIdx.x == B - 1) {
    int h = 0x3fffffff;
    if (x + 1 < cols) h = ASIM_LD(w, GLOBAL_LOAD_DWORD, src + x + 1, 4, 1);
    ASIM_ST(w, DS_WRITE_B32, &prev[B + 1], h, 4, 3);
  }
  ASIM_BARRIER(w);
  if (x < cols) {
    const int l = ASIM_LD(w, DS_READ_B32, &prev[threadIdx.x], 5, 3);
    const int u = ASIM_LD(w, DS_READ_B32, &prev[threadIdx.x + 1], 6, 3);
    const int r = ASIM_LD(w, DS_READ_B32, &prev[threadIdx.x + 2], 7, 3);
    const int wv = ASIM_LD(w, GLOBAL_LOAD_DWORD, wall_row + x, 8, 1);
    ASIM_VALU(w, S_WAITCNT, 0, 0);
    ASIM_VALU(w, V_MIN_F32, 9, 5, 6);
    ASIM_VALU(w, V_MIN_F32, 9, 9, 7);
    ASIM_VALU(w, V_ADD_U32, 10, 9, 8);
    const int m = l < u ? (l < r ? l : r) : (u < r ? u : r);
    ASIM_ST(w, GLOBAL_STORE_DWORD, dst + x, wv + m, 10, 1);
  }
  w.exit();
}

int main(int argc, char** argv) {
  const int cols = argc > 1 ? atoi(argv[1]) : 100000, rows = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> wall((size_t)rows * cols);
  uint32_t s = 12345;
  for (auto& v : wall) {
    s = s * 1664525u + 1013904223u;
    v = (int)((s >> 16) % 10);
  }
  int *dwall, *r0, *r1;
  ASIM_HIP(hipMalloc(&dwall, wall.size() * 4));
  ASIM_HIP(hipMalloc(&r0, cols * 4));
  ASIM_HIP(hipMalloc(&r1, cols * 4));
  memcpy_htod(dwall, wall.data(), wall.size() * 4);
  memcpy_htod(r0, wall.data(), cols * 4);
  const dim3 grid((cols + B - 1) / B), blk(B);
  for (int t = 1; t < rows; ++t)
    launch("_Z14dynproc_kerneliPiS_S_iiii", dynproc<On>, dynproc<Off>, grid, blk, 0, 0,
           (const int*)(dwall + (size_t)t * cols), (const int*)(t % 2 ? r0 : r1), t % 2 ? r1 : r0, cols);
  ASIM_HIP(hipDeviceSynchronize());
  std::vector<int> out(cols);
  ASIM_HIP(hipMemcpy(out.data(), (rows - 1) % 2 ? r1 : r0, cols * 4, hipMemcpyDeviceToHost));
  // host check of the DP
  std::vector<int> a(wall.begin(), wall.begin() + cols), b(cols);
  for (int t = 1; t < rows; ++t) {
    for (int x = 0; x < cols; ++x) {
      int m = a[x];
      if (x > 0) m = std::min(m, a[x - 1]);
      if (x + 1 < cols) m = std::min(m, a[x + 1]);
      b[x] = wall[(size_t)t * cols + x] + m;
    }
    a.swap(b);
  }
  const bool ok = a == out;
  printf("pathfinder cols=%d rows=%d: %s\n", cols, rows, ok ? "PASSED" : "FAILED");
  ASIM_HIP(hipFree(dwall));
  ASIM_HIP(hipFree(r0));
  ASIM_HIP(hipFree(r1));
  return ok ? 0 : 1;
}
