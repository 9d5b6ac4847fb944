// Command-list driver: the equivalent of the reference's accel-sim.out main
// loop (gpu-simulator/main.cc:55-206) re-built around the epoch engines.
#pragma once
#include <chrono>
#include <deque>
#include <fstream>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "debugger.h"
#include "../config/sim_options.h"
#include "../engine/engine.h"
#include "../parallel/linksim.h"
#include "../power/arch_energy.h"
#include "../power/power.h"

namespace asim {

struct KernelResult {
  std::string name;
  uint32_t uid = 0;
  uint64_t start_cycle = 0;
  uint64_t cycles = 0;
  uint64_t insn = 0;        // thread instructions
  uint64_t warp_insn = 0;
  uint32_t n_cta = 0;
  uint32_t cta_per_sm = 0;
  double ipc = 0;
  double occupancy = 0;     // %
  double wall_s = 0;        // wall time spent simulating this kernel
  bool deadlock = false;
  double avg_power_w = 0;
  double sim_time_ns = 0;   // simulated time of the kernel (core cycles at the clock(s) DVFS ran them)
  double avg_clock_mhz = 0;
  uint64_t epochs = 0;      // PDES epochs simulated (one grid barrier each on the GPU engine)
};

struct CollectiveResult {
  std::string op;
  uint64_t bytes = 0;
  int32_t nranks = 1;
  uint64_t cycles = 0;
};

// Callback used by the distributed layer: given a collective command, return
// its duration in core cycles (e.g. measured by exchanging link packets with
// the other simulated GPUs over RCCL).  When unset the analytic model is used.
using CollectiveHook = std::function<uint64_t(const Command&, uint64_t now_cycle)>;

// one kernel or collective in the command window (reference main.cc
// kernels_info + the busy_streams bookkeeping)
enum OpKind : uint8_t { OP_KERNEL = 0, OP_COLL, OP_RECORD, OP_WAIT };
struct StreamOp {
  size_t cmd = 0;             // command index
  OpKind kind = OP_KERNEL;
  uint64_t stream = 0;
  uint64_t event = 0, wait_for = 0;  // event ops: id; wait: records of it that must have fired
  bool queued = false;        // kernel: right behind another kernel (no host sync between)
  uint64_t submit = 0;        // kernel: cycle the host submits it (-sim_host_launch_interval)
  bool after_copy = false;    // kernel: the run's first, behind the initial host copies
  bool launched = false;
  int slot = -1;              // kernel: engine slot while running
  uint64_t start = 0, end = 0;  // launch cycle; collective: completion cycle
  uint64_t start_fs = 0;        // launch time (femtoseconds; the core clock may change under DVFS)
  uint64_t coll_cycles = 0;
  uint64_t epochs = 0;        // engine epochs simulated while the kernel ran
  std::unique_ptr<ReadyKernel> rk;
  KernelDesc kd{};
  // collective with -collective_mem_traffic: the RCCL-style copy kernel that
  // carries its memory traffic (it runs in an engine slot, outside the
  // window) and whether it is still running; the copy kernel's parent
  std::unique_ptr<StreamOp> dma;
  bool dma_pending = false;
  uint64_t dma_end = 0;
  StreamOp* parent = nullptr;
  const char* occ_limiter = "";
  std::chrono::steady_clock::time_point t_admit;
};

class Simulator {
 public:
  // args: accel-sim.out style argument vector (without argv[0])
  explicit Simulator(const std::vector<std::string>& args);
  ~Simulator();

  int run();  // whole command list; returns 0 on success
  // step API: run the command list up to and including command `idx`
  const std::vector<Command>& commands() const { return cmds_; }
  void load_commands() {
    if (cmds_.empty()) cmds_ = parse_commandlist(dopt_.trace_file);
  }
  void run_command(size_t idx);

  const SimCfg& cfg() const { return cfg_; }
  const DriverOpts& dopts() const { return dopt_; }
  OptionRegistry& registry() { return reg_; }
  Engine& engine() { return *eng_; }
  const std::string& output() const { return out_; }
  void set_echo(bool e) { echo_ = e; }
  void set_collective_hook(CollectiveHook h) { coll_hook_ = std::move(h); }

  uint64_t tot_cycle() const { return tot_cycle_; }
  uint64_t tot_insn() const { return tot_insn_; }
  double wall_seconds() const;
  double sim_seconds() const { return sim_s_; }  // time inside the engine only
  const std::vector<KernelResult>& kernels() const { return results_; }
  const std::vector<CollectiveResult>& collectives() const { return colls_; }
  bool deadlock() const { return deadlock_; }
  // analytic collective duration in core cycles
  uint64_t collective_cycles(const Command& c) const;
  // parameters of the packet-level link model (-collective_model packet)
  LinkParams link_params() const;
  // simulated core clock period in picoseconds
  double core_period_ps() const { return (double)cfg_.per_core / 1000.0; }
  // pipeline dump of SM `sm` / channel `ch` (-1: every busy SM / every channel,
  // -2: none), decoded from the engine state image (reference dump_pipeline)
  std::string dump_pipeline(int sm, int ch);

 private:
  void print(const char* fmt, ...);
  // stream window (main.cc:74-197)
  size_t window_size() const;
  void admit(size_t end);                 // move commands [next_cmd_, end) into the window
  void run_now(const Command& c);         // memcpy / communicator bookkeeping
  void admit_kernel(size_t idx);
  void setup_kernel_op(StreamOp& op, bool apply_cta_cap);
  void launch_collective_dma(StreamOp& coll);
  void launch_ready();
  void launch_collective(StreamOp& op);
  void step();                            // run to the next kernel / collective completion
  void retire_collectives();
  void finish_kernel(uint32_t slot, const RunResult& rr);
  void check_limits();
  // host trace prefetch (the reference's TODO, AS/main.cc:25-44): the next
  // kernel's trace is parsed and coalesced on a worker thread while the
  // engine simulates
  void prefetch_next();
  std::unique_ptr<ReadyKernel> take_kernel(size_t idx);
  bool stream_from_host(const std::string& path) const;
  // trace ingest: HIP device of the GPU engine (-1: host coalescer) and what
  // ran where (the prefetch thread adds to it too; declared before pf_ so that
  // pending prefetches finish before these are destroyed)
  int ingest_dev_ = -1;
  std::mutex ingest_mu_;
  IngestStats ingest_st_;
  uint64_t ingest_small_ = 0;  // kernels below -gpu_ingest_min_insts
  std::unique_ptr<ReadyKernel> ingest(const HostKernel& k);
  std::map<size_t, std::future<std::unique_ptr<ReadyKernel>>> pf_;
  void print_kernel_stats(const KernelResult& r, const std::vector<SMStats>& sm, const std::vector<MemStats>& mem);
  void print_sim_time();
  // timing-state checkpoint at a kernel boundary / resume from one (returns first command to run)
  std::string checkpoint_file(uint32_t kernel) const;
  void write_checkpoint(size_t cmd_index);
  size_t resume_checkpoint();
  uint32_t kernels_done_ = 0;
  // run in gpu_stat_sample_freq slices, one power sample per slice
  RunResult run_sampled(const RunLimits& lim);

  OptionRegistry reg_;
  SimCfg cfg_{};
  DriverOpts dopt_;
  std::unique_ptr<Engine> eng_;
  std::unique_ptr<PowerModel> power_;
  PowerTracker ptrack_;
  // DVFS governor state: the nominal core period and the current clock ratio
  uint64_t per_core_nom_ = 0;
  double dvfs_ratio_ = 1.0;
  void set_clock_ratio(double ratio);
  std::unique_ptr<std::ofstream> power_report_, power_trace_, power_steady_, visualizer_;
  // drain the engine's debug trace events, print the streams the user asked
  // for, return all of them (the debugger evaluates its breakpoints on them)
  std::vector<TraceEv> emit_trace();
  uint32_t print_mask_ = 0;   // trace streams to print (-trace_components)
  int32_t print_sm_ = -1, print_mem_ = -1;  // units to print (the debugger records all)
  std::unique_ptr<Debugger> dbg_;
  bool dbg_quit_ = false;
  void write_visualizer_sample(const std::string& kname, uint64_t now, uint64_t cycles,
                               const std::vector<SMStats>& dsm, const std::vector<MemStats>& dm);
  std::vector<Command> cmds_;
  std::string out_;
  bool echo_ = true;
  CollectiveHook coll_hook_;
  uint64_t tot_cycle_ = 0, tot_insn_ = 0, tot_warp_insn_ = 0;
  uint64_t tot_cta_ = 0;
  std::vector<SMStats> prev_sm_;
  std::vector<MemStats> prev_mem_;
  std::vector<KernelResult> results_;
  std::vector<CollectiveResult> colls_;
  std::chrono::steady_clock::time_point t_start_;
  double sim_s_ = 0;
  bool deadlock_ = false;
  uint32_t next_uid_ = 1;
  // command window: kernels / collectives admitted and not yet completed
  std::deque<std::unique_ptr<StreamOp>> win_;
  size_t kernels_in_window() const;
  std::map<uint64_t, uint64_t> ev_admitted_, ev_fired_;  // per event: records admitted / fired
  StreamOp* slot_op_[kMaxConc] = {};  // running kernel per engine slot
  size_t next_cmd_ = 0;
  bool stop_ = false;
  bool ckpt_pending_ = false;
  bool last_cmd_kernel_ = false;  // the previous admitted command was a kernel launch
  uint64_t host_t_ = 0;           // host model: cycle of the host's next kernel submission
  bool copy_since_kernel_ = false;  // a host memcpy ran since the last kernel was admitted
  bool any_kernel_admitted_ = false;
  uint64_t dma_count_ = 0;        // collective copy kernels launched
  uint64_t pwr_in_loop_samples_ = 0;  // power samples the engine took inside its cycle loop
  uint64_t host_streamed_ = 0;    // kernels read per CTA from their files (-trace_host_budget_mb)
  uint64_t host_stream_peak_ = 0;  // largest host trace footprint of one of them
  bool cap_hit_ = false;  // a run cap (-gpgpu_max_insn / _max_cta / _max_completed_cta) stopped a kernel
};

}  // namespace asim
