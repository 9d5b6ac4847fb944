// Load-to-use latency of the memory hierarchy by footprint (reference
// GPU_Microbenchmark l1_cache/l1_lat, l2_cache/l2_lat, mem/mem_lat): one lane
// pointer-chases a random cyclic permutation; footprints below the vL1D
// (32 KB), inside one XCD's L2 (4 MB), inside the Infinity Cache (MALL) and
// far beyond it give the four plateaus.
#include "ubench.h"

int main(int argc, char** argv) {
  UbDevice d;
  const int iters = 4096;
  struct Pt {
    size_t bytes;
    double ticks;
  };
  std::vector<Pt> pts;
  // the last point touches 4 GB of distinct lines: 16x the 256 MB MALL
  for (size_t kb : {4, 8, 16, 24, 64, 256, 1024, 2048, 3072, 16384, 65536, 131072, 4194304}) {
    const size_t bytes = kb * 1024;
    const size_t stride = 128;
    pts.push_back({bytes, ub_chase_latency(bytes, stride, iters)});
    printf("chase %8zu KB stride %4zu B : %7.1f cycles/load\n", kb, stride, pts.back().ticks);
  }
  auto at = [&](size_t kb) {
    for (auto& p : pts)
      if (p.bytes == kb * 1024) return p.ticks;
    return 0.0;
  };
  const double l1 = at(8), l2 = at(1024), mall = at(65536), hbm = at(4194304);
  printf("# l1 %.0f  l2 %.0f  mall %.0f  hbm %.0f cycles\n", l1, l2, mall, hbm);
  ub_opt("-gpgpu_l1_latency", (long long)(l1 + 0.5));
  // The simulator's L2 stands for the per-XCD L2 that a kernel's re-used
  // lines hit (its hit costs the XCD-L2 latency, split as gpgpu-sim does into
  // the L1 miss path, two icnt traversals and the ROP delay), and an L2 miss
  // for the memory-side Infinity Cache (MALL) that holds freshly copied data
  // (hipMemcpy'd inputs of ordinary working sets sit there), so the DRAM
  // latency is the MALL-over-L2 step.  Streams beyond the 256 MB MALL pay the
  // HBM latency on hardware; that step is reported only.
  ub_opt("-gpgpu_l2_rop_latency", (long long)std::max(1.0, l2 - l1 - 16));
  ub_opt("-dram_latency", (long long)std::max(1.0, mall - l2));
  printf("# hbm_over_mall_latency %.0f\n", hbm - mall);
  printf("# mall_hit_latency %.0f\n# xcd_l2_hit_latency %.0f\n", mall, l2);
  return 0;
}
