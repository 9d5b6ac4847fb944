// Fill granularity of the vector L1 and of the L2 (reference GPU_Microbenchmark
// l1_cache/l1_access_grain, l1_sector and l2_cache/l2_access_grain): one lane
// loads byte offset 0 of a cold line, then byte offset `off` of the same line,
// and times the second load.  If the first miss filled the part of the line
// holding `off`, the second load hits (L1 latency); if the cache fills per
// sector, an offset in another 32-byte sector misses again.  For the L2 the
// L1 copy is first evicted by streaming through 2x the L1 capacity, so the
// second load can only hit in the L2.  Prints the fill granules and the
// sectored / non-sectored letter of the -gpgpu_cache:dl1 / dl2 options.
#include "ubench.h"

__global__ void ub_grain_kernel(const int* __restrict__ line, const int* __restrict__ evict, int evict_n, int off_ints,
                                uint64_t* out) {
  if (threadIdx.x != 0) return;
  const int* p = line;
  asm volatile("" : "+v"(p));
  int a = p[0];                       // cold miss: HBM -> L2 -> L1
  __builtin_amdgcn_s_waitcnt(0);
  int sink = 0;
  for (int i = 0; i < evict_n; i += 32) sink += evict[i];  // optional L1 eviction sweep
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t0 = ub_clock();
  int b = p[off_ints];
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t1 = ub_clock();
  out[0] = t1 - t0;
  out[1] = (uint64_t)(a + b + sink);
}

static double probe(int* lines, int* evict, int evict_n, int off_bytes, int trials, uint64_t* o) {
  std::vector<double> v;
  for (int t = 0; t < trials; ++t) {
    int* line = lines + (size_t)t * 4096;  // a fresh line (16 KB apart) per trial
    hipLaunchKernelGGL(ub_grain_kernel, dim3(1), dim3(64), 0, 0, line, evict, evict_n, off_bytes / 4, o);
    UB_CHECK(hipDeviceSynchronize());
    uint64_t r[2];
    UB_CHECK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
    v.push_back((double)r[0]);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  UbDevice d;
  const int trials = 32, offs[] = {4, 16, 32, 64, 96, 124};
  int *lines, *evict;
  uint64_t* o;
  const size_t nlines = (size_t)trials * 2 * 10;  // fresh lines for every (offset, level) trial
  UB_CHECK(hipMalloc(&lines, nlines * 4096 * sizeof(int)));
  UB_CHECK(hipMemset(lines, 0, nlines * 4096 * sizeof(int)));
  const int evict_n = 2 * 64 * 1024 / 4;  // 2x a 64 KB L1 in ints (one load per 128 B)
  UB_CHECK(hipMalloc(&evict, (size_t)evict_n * sizeof(int)));
  UB_CHECK(hipMemset(evict, 0, (size_t)evict_n * sizeof(int)));
  UB_CHECK(hipMalloc(&o, 16));
  size_t slot = 0;
  auto next = [&]() { return lines + (slot++) * 4096 * trials; };
  // references in the same kernel shape (the stamps' own cost included):
  // the same word again (an L1 hit) and the same word after the L1 sweep
  // (an L2 hit); a word of another sector / line is classified against them
  const double hit = probe(next(), evict, 0, 0, trials, o);
  const double l2hit = probe(next(), evict, evict_n, 0, trials, o);
  printf("# timed_l1_hit %.0f\n# timed_l2_hit %.0f\n", hit, l2hit);
  int l1_grain = 128, l2_grain = 128;
  bool l1_done = false, l2_done = false;
  for (int off : offs) {
    const double a = probe(next(), evict, 0, off, trials, o);
    const double b = probe(next(), evict, evict_n, off, trials, o);
    const bool l1_hit = a < 0.5 * (hit + l2hit), l2_hit = b < l2hit + 0.5 * (l2hit - hit) + 50;
    printf("second load at +%3d B: %6.0f cycles (%s in L1), after L1 eviction %6.0f cycles (%s in L2)\n", off, a,
           l1_hit ? "hit" : "miss", b, l2_hit ? "hit" : "miss");
    if (!l1_hit && !l1_done) { l1_grain = off < 32 ? 32 : (off / 32) * 32; l1_done = true; }
    if (!l2_hit && !l2_done) { l2_grain = off < 32 ? 32 : (off / 32) * 32; l2_done = true; }
  }
  printf("# l1_fill_granule_bytes %d\n# l2_fill_granule_bytes %d\n", l1_grain, l2_grain);
  printf("# l1_sectored %d\n# l2_sectored %d\n", l1_grain < 128 ? 1 : 0, l2_grain < 128 ? 1 : 0);
  UB_CHECK(hipFree(lines));
  UB_CHECK(hipFree(evict));
  UB_CHECK(hipFree(o));
  return 0;
}
