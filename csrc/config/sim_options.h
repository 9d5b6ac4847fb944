// gpgpusim.config / trace.config option set and its translation into the
// POD SimCfg consumed by the cycle model.
#pragma once
#include <string>
#include <vector>

#include "../model/config.h"
#include "options.h"

namespace asim {

// Registers every option the reference simulator accepts in trace mode
// (gpu-sim.cc:101-763, shader/memory/power/icnt/ptx/trace registrations; ~250
// flags incl. the looped -specialized_unit_N and
// -trace_opcode_latency_initiation_spec_op_N) plus this simulator's own
// extensions (prefixed -sim_ / -icnt_latency / -rccl_*).  PTX-only flags are
// accepted and ignored, as tested configs still carry them.
void register_sim_options(OptionRegistry& r);

// Options that are accepted for config-file compatibility but change nothing
// in this simulator, set by the user to a value other than their default: one
// message per option, naming why (PTX-mode only, not modelled, ...).  The
// driver prints them as warnings so a config never silently loses an effect.
std::vector<std::string> unmodelled_option_warnings(const OptionRegistry& r);

// Derive the model configuration.  Throws OptionError on malformed composite
// strings or configurations beyond the compiled capacity caps.
SimCfg derive_sim_cfg(const OptionRegistry& r);

// cache geometry string  <S|N>:<sets>:<line>:<assoc>,<rep>:<wr>:<alloc>:<wr_alloc>:<idx>,<mshr>:<N>:<merge>,<mq>[:...]
CacheGeom parse_cache_geom(const std::string& s, bool any_line = false);

struct KernelShape {
  uint32_t threads_per_cta;
  uint32_t shmem_per_cta;
  uint32_t regs_per_thread;
  uint32_t n_cta;
};
// resource-limited CTAs per SM and adaptive L1 geometry (reference
// shader_core_config::max_cta, shader.cc:3476-3588)
struct Occupancy {
  uint32_t cta_per_sm;
  uint32_t l1_sets;
  uint32_t l1_assoc;
  uint32_t shmem_kb;  // carve-out chosen by the adaptive config
  const char* limiter;
};
Occupancy compute_occupancy(const SimCfg& c, const KernelShape& k);

// extra: option values that are not part of SimCfg but used by the driver
struct DriverOpts {
  std::string trace_file;
  int64_t max_cycle = 0;
  int64_t max_insn = 0;
  int32_t max_cta = 0;
  int32_t max_completed_cta = 0;
  bool flush_l1 = false;
  bool sqc_invalidate = false;  // -sim_sqc_invalidate_at_launch
  bool flush_l2 = false;
  bool l2_kernel_release = false;
  bool coll_mem_traffic = false;   // -collective_mem_traffic: collectives run a copy kernel
  uint64_t host_launch_interval = 0;      // -sim_host_launch_interval (cycles)
  uint64_t first_kernel_latency = 0;      // -sim_first_kernel_latency (cycles)
  bool copy_latency_every = false;        // -sim_copy_latency_every_kernel: ... for every kernel behind a copy
  uint64_t kernel_min_cycles_queued = 0;  // -sim_kernel_min_cycles_queued
  bool dvfs = false;               // -dvfs_enabled: the power-cap DVFS governor
  double dvfs_min_clock_ratio = 0.5;  // -sim_l2_kernel_release: write back + invalidate the L2s at kernel end
  bool deadlock_detect = true;
  int32_t nccl_allreduce_latency = 100;
  std::string collective_model;   // const | ring | tree | packet
  double xgmi_link_gbps = 153.0;
  double xgmi_latency_ns = 1000.0;
  uint32_t xgmi_links = 7;
  uint32_t coll_slice_bytes = 131072;
  uint32_t coll_max_channels = 16;
  double coll_reduce_gbps = 900.0;
  int32_t concurrent_kernel_sm = 0;
  int32_t max_concurrent_kernel = 32;
  bool power_enabled = false;
  std::string power_xml;
  int32_t power_mode = 0;
  std::string hw_perf_file;
  std::string hw_perf_bench;
  bool hybrid_use_sim[17] = {};   // indexed by asim::HwCounter
  bool power_trace = false;
  bool steady_power = false;
  double steady_dev_pct = 8;
  uint32_t steady_samples = 4;
  std::string power_report_file;
  int32_t memlatency_stat = 0;     // -gpgpu_memlatency_stat: print memory latency statistics
  bool visualizer = false;         // -visualizer_enabled: per-sample activity log
  std::string visualizer_file;
  // timing-state checkpoint / resume at kernel boundaries (trace mode)
  int32_t checkpoint_option = 0, checkpoint_kernel = 1;
  int32_t resume_option = 0, resume_kernel = 0;
  std::string checkpoint_dir;
  uint64_t stat_sample_freq = 500;
  std::string engine;             // cpu | gpu | check
  uint64_t check_interval = 4096;  // -sim_engine check
  std::string check_primary = "gpu";
  uint64_t check_corrupt_at = 0;
  uint32_t check_corrupt_mailbox = 0;
  bool trace_enabled = false;
  std::string trace_components;
  int32_t trace_sampling_core = 0;
  uint32_t sim_epochs_per_launch = 4096;
  bool gpu_ingest = true;      // -gpu_ingest: coalesce traces on the GPU engine's device
  uint64_t gpu_ingest_min = 32768;  // -gpu_ingest_min_insts: smaller kernels stay on the host
  bool power_in_loop = true;  // -power_in_loop: engines sample power inside their cycle loop
  double host_budget_mb = 0;  // -trace_host_budget_mb: stream larger text traces per CTA (0 = off)
  bool trace_prefetch = true;  // -trace_prefetch: parse the next kernel while this one simulates
  // interactive timing debugger (csrc/driver/debugger.h)
  bool debug = false;
  std::string debug_script;
  uint64_t debug_step = 0;
  uint64_t break_cycle = 0;
};
DriverOpts derive_driver_opts(const OptionRegistry& r);

}  // namespace asim
