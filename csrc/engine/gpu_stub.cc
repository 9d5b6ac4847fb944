// Linked into CPU-only builds (no HIP engine object).
#include "engine.h"

namespace asim {
std::unique_ptr<Engine> make_gpu_engine() { return nullptr; }
bool gpu_engine_available() { return false; }
}  // namespace asim

namespace asim {
int gpu_cu_count() { return 0; }
int gpu_cus_per_sim(uint32_t n_sm, uint32_t n_mem) { return (int)(n_sm + n_mem); }
std::map<std::string, uint64_t> gpu_pool_stats() { return {}; }
void gpu_pool_trim() {}
std::map<std::string, uint64_t> gpu_batch_stats() { return {}; }
std::map<std::string, std::map<std::string, uint64_t>> gpu_engine_modes() { return {}; }
EngineKernelInfo gpu_engine_kernel_info() { return EngineKernelInfo{}; }
}  // namespace asim

namespace asim {
bool gpu_coalesce_kernel(const HostKernel&, const SimCfg&, int, ReadyKernel&, IngestStats*) { return false; }
}  // namespace asim

namespace asim {
int gpu_current_device() { return -1; }
}  // namespace asim
