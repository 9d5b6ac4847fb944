// Device configuration -> gpgpusim.config core/memory lines (reference
// GPU_Microbenchmark core/config_* and mem/config_dram programs: print the
// -gpgpu_* options derived from the device properties).
#include "ubench.h"

int main() {
  UbDevice d;
  const hipDeviceProp_t& p = d.p;
  const double mhz = ub_shader_mhz();
  std::string name = p.name;
  if (name.empty()) name = std::string(p.gcnArchName).rfind("gfx950", 0) == 0 ? "AMD Instinct MI355X" : "AMD GPU";
  printf("# device: %s (%s), %d CUs, warp %d, LDS/CU %zu KB, L2 %d KB, HBM bus %d bit @ %.0f MHz\n", name.c_str(),
         p.gcnArchName, p.multiProcessorCount, p.warpSize, p.sharedMemPerMultiprocessor / 1024, p.l2CacheSize / 1024,
         p.memoryBusWidth, p.memoryClockRate / 1000.0);
  printf("# shader clock: reported %.0f MHz, measured %.0f MHz\n", p.clockRate / 1000.0, mhz);
  const int cus = p.multiProcessorCount;
  ub_opt("-gpgpu_n_clusters", cus);
  ub_opt("-gpgpu_n_cores_per_cluster", 1);
  ub_opt("-gpgpu_shader_core_pipeline",
         std::to_string(p.maxThreadsPerMultiProcessor) + ":" + std::to_string(p.warpSize));
  ub_opt("-gpgpu_shader_registers", (long long)p.regsPerMultiprocessor);
  ub_opt("-gpgpu_registers_per_block", (long long)p.regsPerBlock);
  ub_opt("-gpgpu_shmem_size", (long long)p.sharedMemPerMultiprocessor);
  ub_opt("-gpgpu_shmem_per_block", (long long)p.sharedMemPerBlock);
  ub_opt("-gpgpu_shader_cta", (long long)std::min(32, p.maxThreadsPerMultiProcessor / 64));
  // HBM3E: 8 stacks x 16 channels of 64 bits; one simulated channel (with
  // one L2 slice) per 64-bit channel
  const int channels = std::max(1, p.memoryBusWidth / 64);
  ub_opt("-gpgpu_n_mem", channels);
  ub_opt("-gpgpu_n_sub_partition_per_mchannel", 1);
  const double mem_mhz = p.memoryClockRate / 1000.0;
  // -gpgpu_dram_buswidth comes from ub_mem_bw (sized to the measured bandwidth)
  char clk[128];
  snprintf(clk, sizeof(clk), "%.1f:%.1f:%.1f:%.1f", mhz > 0 ? mhz : p.clockRate / 1000.0,
           mhz > 0 ? mhz : p.clockRate / 1000.0, mhz > 0 ? mhz : p.clockRate / 1000.0, mem_mhz);
  ub_opt("-gpgpu_clock_domains", clk);
  // L2: hipDeviceProp reports one XCD's L2; the chip has 8 XCDs.  The
  // simulator's memory-side L2 gets the chip total, split across the
  // memory sub-partitions (16-way, 128B lines).  Line-granular ('N'): an
  // L2 miss fills the whole 128 B line (rocprofv3 TCC_EA0_RDREQ_128B carries
  // almost all of the fill traffic of the Rodinia suite, profiles/correlation)
  const long long l2_bytes = (long long)p.l2CacheSize * 8;
  const long long per_sub = std::max<long long>(128 * 16, l2_bytes / channels);
  const long long sets = std::max<long long>(1, per_sub / (128 * 16));
  ub_opt("-gpgpu_cache:dl2", "N:" + std::to_string(sets) + ":128:16,L:B:m:L:P,A:192:4,32:0,32");
  // CDNA (gfx9): each SIMD has one VALU port that INT, FP64 and
  // transcendental work issue on (no separate INT / SFU pipes)
  if (std::string(p.gcnArchName).rfind("gfx9", 0) == 0) ub_opt("-sim_single_valu", 1);
  printf("# measured_shader_mhz %.1f\n", mhz);
  return 0;
}
