#include "simulator.h"

#include <sys/stat.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <filesystem>
#include <stdexcept>

namespace asim {

// out = a - b for POD stat vectors of 64-bit counters (b empty = zeros)
template <class T>
static void stat_delta(const std::vector<T>& a, const std::vector<T>& b, std::vector<T>& out) {
  static_assert(sizeof(T) % 8 == 0, "stat structs are arrays of 64-bit counters");
  out.resize(a.size());
  for (size_t i = 0; i < a.size(); ++i) {
    const uint64_t* x = (const uint64_t*)&a[i];
    uint64_t* o = (uint64_t*)&out[i];
    if (i < b.size()) {
      const uint64_t* y = (const uint64_t*)&b[i];
      for (size_t k = 0; k < sizeof(T) / 8; ++k) o[k] = x[k] - y[k];
    } else {
      for (size_t k = 0; k < sizeof(T) / 8; ++k) o[k] = x[k];
    }
  }
}

Simulator::Simulator(const std::vector<std::string>& args) {
  t_start_ = std::chrono::steady_clock::now();
  register_sim_options(reg_);
  reg_.parse_cmdline(args, false);
  cfg_ = derive_sim_cfg(reg_);
  dopt_ = derive_driver_opts(reg_);
  if (dopt_.engine == "gpu") {
    eng_ = make_gpu_engine();
    if (!eng_) throw std::runtime_error("-sim_engine gpu requested but the HIP engine is unavailable");
    if (dopt_.gpu_ingest) ingest_dev_ = gpu_current_device();
  } else if (dopt_.engine == "cpu") {
    eng_ = make_cpu_engine();
  } else if (dopt_.engine == "check") {
    std::unique_ptr<Engine> primary;
    if (dopt_.check_primary == "gpu") {
      primary = make_gpu_engine();
      if (!primary) throw std::runtime_error("-sim_engine check: the HIP engine is unavailable");
    } else if (dopt_.check_primary == "cpu") {
      primary = make_cpu_engine();
    } else {
      throw OptionError("-sim_check_primary must be cpu or gpu");
    }
    eng_ = make_check_engine(std::move(primary), make_cpu_engine(), dopt_.check_interval, dopt_.check_corrupt_at,
                             dopt_.check_corrupt_mailbox != 0);
  } else {
    throw OptionError("-sim_engine must be cpu, gpu or check");
  }
  print_mask_ = cfg_.trace_mask;
  if (dopt_.debug) {
    // the debugger evaluates breakpoints / watchpoints on the engine's trace
    // events: record the streams it needs (printed only if also requested)
    cfg_.trace_mask |= Debugger::trace_mask();
    // every unit records (breakpoints may name any SM); what is printed still
    // follows -trace_sampling_core / _memory_partition
    print_sm_ = cfg_.trace_sm;
    print_mem_ = cfg_.trace_mem;
    cfg_.trace_sm = -1;
    cfg_.trace_mem = -1;
    Debugger::Hooks h;
    h.print = [this](const std::string& s) { print("%s", s.c_str()); };
    h.dump = [this](int sm, int ch) { return dump_pipeline(sm, ch); };
    h.status = [this]() {
      char b[200];
      snprintf(b, sizeof(b), "cycle %llu, kernels completed %zu, thread instructions of completed kernels %llu",
               (unsigned long long)eng_->now(), results_.size(), (unsigned long long)tot_insn_);
      return std::string(b);
    };
    dbg_.reset(new Debugger(dopt_.debug_script, dopt_.break_cycle, h));
  }
  eng_->init(cfg_);
  per_core_nom_ = cfg_.per_core;
  if (dopt_.power_enabled) {
    power_.reset(new PowerModel());
    std::string err;
    if (!power_->load_xml(dopt_.power_xml, &err)) throw std::runtime_error("power model: " + err);
    // the governor never goes below what the engine's buffers were sized for
    power_->set_param("dvfs_min_clock_ratio",
                      std::max(power_->param("dvfs_min_clock_ratio", 0.0), dopt_.dvfs_min_clock_ratio));
    power_report_.reset(new std::ofstream(dopt_.power_report_file));
    if (!*power_report_) throw std::runtime_error("cannot write " + dopt_.power_report_file);
    if (power_->param("energy_model", 0.0) >= 1.0) {
      // per-access energies from this machine's geometry (McPAT / CACTI role)
      ArchEnergyParams ap;
      ap.node_nm = power_->param("core_tech_node", ap.node_nm);
      ap.vdd = power_->param("core_vdd", 0.0);
      ap.dram_pj_per_bit = power_->param("dram_pj_per_bit", ap.dram_pj_per_bit);
      ap.dram_act_nj = power_->param("dram_act_nj", ap.dram_act_nj);
      ap.tensor_macs_per_lane = power_->param("tensor_macs_per_lane", 0.0);
      const ArchEnergy ae = arch_energy(cfg_, ap);
      power_->set_base(ae.base_nj);
      *power_report_ << "architectural energy model (energy_model = 1)\n" << arch_energy_report(ae) << "\n";
    }
    if (dopt_.power_trace) {
      power_trace_.reset(new std::ofstream("accelwattch_power_trace.csv"));
      ptrack_.write_trace_header(*power_trace_);
    }
    if (dopt_.steady_power) {
      power_steady_.reset(new std::ofstream("accelwattch_steady_state.csv"));
      *power_steady_ << "kernel,start_cycle,end_cycle,samples,avg_power\n";
      ptrack_.set_steady(dopt_.steady_dev_pct, dopt_.steady_samples);
    }
  }
  if (dopt_.visualizer) {
    visualizer_.reset(new std::ofstream(dopt_.visualizer_file));
    if (!*visualizer_) throw std::runtime_error("cannot write " + dopt_.visualizer_file);
  }
}

Simulator::~Simulator() = default;

void Simulator::print(const char* fmt, ...) {
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n < 0) return;
  std::string s;
  if ((size_t)n < sizeof(buf)) {
    s.assign(buf, (size_t)n);
  } else {  // long message (pipeline dumps): format again into a sized buffer
    s.resize((size_t)n + 1);
    va_start(ap, fmt);
    vsnprintf(&s[0], s.size(), fmt, ap);
    va_end(ap);
    s.resize((size_t)n);
  }
  out_ += s;
  if (echo_) {
    fputs(s.c_str(), stdout);
  }
}

double Simulator::wall_seconds() const {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start_).count();
}

// The command loop (reference gpu-simulator/main.cc:74-197): commands enter
// a window in trace order -- up to -gpgpu_max_concurrent_kernel kernels /
// collectives with -gpgpu_concurrent_kernel_sm, else one -- memcpys are
// applied as they are reached, and a windowed operation starts once every
// earlier operation of its stream has finished (stream order; kernels also
// need a free engine slot).  The engine then runs until the next kernel or
// collective completes.
int Simulator::run() {
  print("Accel-Sim-AMD [MI355X-native trace-driven simulator, engine=%s]\n", eng_->name());
  for (const std::string& w : unmodelled_option_warnings(reg_)) print("GPGPU-Sim: %s\n", w.c_str());
  cmds_ = parse_commandlist(dopt_.trace_file);
  next_cmd_ = 0;
  if (dopt_.resume_option) next_cmd_ = resume_checkpoint();
  while (!stop_ && (next_cmd_ < cmds_.size() || !win_.empty())) {
    admit(cmds_.size());
    step();
  }
  print("GPGPU-Sim: *** simulation thread exiting ***\n");
  print("GPGPU-Sim: *** exit detected ***\n");
  fflush(stdout);
  return deadlock_ ? 1 : 0;
}

size_t Simulator::window_size() const {
  return dopt_.concurrent_kernel_sm ? std::max<uint32_t>(1, cfg_.max_concurrent_kernel) : 1;
}

size_t Simulator::kernels_in_window() const {
  size_t n = 0;
  for (auto& op : win_) n += op->kind == OP_KERNEL ? 1 : 0;
  return n;
}

// Serially (no -gpgpu_concurrent_kernel_sm) the window holds one operation of
// any kind; with concurrent kernels it bounds the kernels, and collectives /
// events ride along in trace order.
void Simulator::admit(size_t end) {
  bool admitted = false;  // a windowed operation entered the window in this pass
  while (next_cmd_ < end) {
    const Command& c = cmds_[next_cmd_];
    const bool windowed = c.type == CMD_KERNEL || c.type == CMD_COLLECTIVE || c.type == CMD_EVENT_RECORD ||
                          c.type == CMD_EVENT_WAIT;
    if (windowed) {
      const bool full = dopt_.concurrent_kernel_sm ? (c.type == CMD_KERNEL && kernels_in_window() >= window_size())
                                                   : win_.size() >= window_size();
      if (full) break;
    } else if (c.type == CMD_MEMCPY_HTOD || c.type == CMD_MEMCPY_DTOH) {
      // A memcpy behind a kernel is reached only after the engine has run
      // (reference main.cc:83-161: each pass of the command loop admits one
      // group, then simulates until a kernel completes): serially it waits
      // for the window to drain, with concurrent kernels for the next
      // completion.  Applying it earlier would pre-fill the L2 under a kernel
      // that has not been simulated yet.
      if (dopt_.concurrent_kernel_sm ? admitted : !win_.empty()) break;
    }
    const size_t i = next_cmd_++;
    if (windowed) admitted = true;
    if (c.type == CMD_KERNEL) {
      admit_kernel(i);
      win_.back()->queued = last_cmd_kernel_;
      // host model: launches leave the host -sim_host_launch_interval cycles
      // apart (the host resumes at the engine's clock after a sync)
      win_.back()->submit = host_t_;
      host_t_ += dopt_.host_launch_interval;
      win_.back()->after_copy = copy_since_kernel_ && (dopt_.copy_latency_every || !any_kernel_admitted_);
      copy_since_kernel_ = false;
      any_kernel_admitted_ = true;
      last_cmd_kernel_ = true;
    } else if (windowed) {
      std::unique_ptr<StreamOp> op(new StreamOp());
      op->cmd = i;
      op->stream = c.stream;
      op->event = c.event;
      if (c.type == CMD_COLLECTIVE) {
        op->kind = OP_COLL;
      } else if (c.type == CMD_EVENT_RECORD) {
        op->kind = OP_RECORD;
        ev_admitted_[c.event]++;
      } else {
        op->kind = OP_WAIT;
        op->wait_for = ev_admitted_[c.event];  // the latest record issued before the wait
      }
      win_.push_back(std::move(op));
    } else {
      if (c.type == CMD_MEMCPY_HTOD || c.type == CMD_MEMCPY_DTOH) {
        last_cmd_kernel_ = false;  // host sync
        copy_since_kernel_ = true;
        host_t_ = std::max(host_t_, eng_->now());
      }
      run_now(c);
    }
  }
}

void Simulator::run_now(const Command& c) {
  switch (c.type) {
    case CMD_MEMCPY_HTOD:
      print("launching memcpy command : %s\n", c.text.c_str());
      if (cfg_.perf_memcpy) eng_->memcpy_fill_l2(c.addr, c.bytes);
      break;
    case CMD_COLL_INIT:
    case CMD_COLL_DESTROY:
    case CMD_GROUP_START:
    case CMD_GROUP_END:
      print("%s was run!\n", c.text.c_str());
      break;
    default:
      break;
  }
}

// step API: run the command list up to and including command `idx` (the
// window drains, so every admitted kernel / collective completes)
void Simulator::run_command(size_t idx) {
  if (cmds_.empty()) cmds_ = parse_commandlist(dopt_.trace_file);
  if (next_cmd_ < idx) next_cmd_ = idx;
  const size_t end = std::min(idx + 1, cmds_.size());
  while (!stop_ && (next_cmd_ < end || !win_.empty())) {
    admit(end);
    if (!win_.empty()) step();
  }
}

// Checkpoint file: magic, driver counters, previous stat snapshots, engine image.
namespace {
struct CkptHeader {
  uint64_t magic = 0x41534d434b505432ull;  // "ASMCKPT2"
  uint64_t cmd_index = 0, kernels_done = 0;
  uint64_t tot_cycle = 0, tot_insn = 0, tot_warp_insn = 0, tot_cta = 0, next_uid = 0;
  uint64_t n_sm_stats = 0, n_mem_stats = 0, engine_bytes = 0;
  uint64_t per_core = 0, clk_base_cyc = 0, clk_base_fs = 0;  // the core-clock time base (DVFS)
};
}  // namespace

std::string Simulator::checkpoint_file(uint32_t kernel) const {
  return dopt_.checkpoint_dir + "/asim_state_kernel" + std::to_string(kernel) + ".ckpt";
}

void Simulator::write_checkpoint(size_t cmd_index) {
  std::vector<uint8_t> eng;
  eng_->save_state(eng);
  CkptHeader h;
  h.cmd_index = cmd_index;
  h.kernels_done = kernels_done_;
  h.tot_cycle = tot_cycle_;
  h.tot_insn = tot_insn_;
  h.tot_warp_insn = tot_warp_insn_;
  h.tot_cta = tot_cta_;
  h.next_uid = next_uid_;
  h.n_sm_stats = prev_sm_.size();
  h.n_mem_stats = prev_mem_.size();
  h.engine_bytes = eng.size();
  h.per_core = cfg_.per_core;
  h.clk_base_cyc = cfg_.clk_base_cyc;
  h.clk_base_fs = cfg_.clk_base_fs;
  {
    std::error_code ec;
    std::filesystem::create_directories(dopt_.checkpoint_dir, ec);
    if (ec) throw std::runtime_error("cannot create " + dopt_.checkpoint_dir + ": " + ec.message());
  }
  const std::string path = checkpoint_file(kernels_done_);
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write checkpoint " + path);
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && (!h.n_sm_stats || fwrite(prev_sm_.data(), sizeof(SMStats), h.n_sm_stats, f) == h.n_sm_stats);
  ok = ok && (!h.n_mem_stats || fwrite(prev_mem_.data(), sizeof(MemStats), h.n_mem_stats, f) == h.n_mem_stats);
  ok = ok && fwrite(eng.data(), 1, eng.size(), f) == eng.size();
  ok = fclose(f) == 0 && ok;
  if (!ok) throw std::runtime_error("short write to checkpoint " + path);
  print("GPGPU-Sim: checkpoint after kernel %u written to %s\n", kernels_done_, path.c_str());
}

size_t Simulator::resume_checkpoint() {
  const std::string path = checkpoint_file((uint32_t)dopt_.resume_kernel);
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open checkpoint " + path);
  CkptHeader h, want;
  bool ok = fread(&h, sizeof(h), 1, f) == 1 && h.magic == want.magic;
  if (!ok) {
    fclose(f);
    throw std::runtime_error("not a checkpoint file: " + path);
  }
  prev_sm_.resize(h.n_sm_stats);
  prev_mem_.resize(h.n_mem_stats);
  std::vector<uint8_t> eng(h.engine_bytes);
  ok = (!h.n_sm_stats || fread(prev_sm_.data(), sizeof(SMStats), h.n_sm_stats, f) == h.n_sm_stats) &&
       (!h.n_mem_stats || fread(prev_mem_.data(), sizeof(MemStats), h.n_mem_stats, f) == h.n_mem_stats) &&
       fread(eng.data(), 1, eng.size(), f) == eng.size();
  fclose(f);
  if (!ok) throw std::runtime_error("truncated checkpoint " + path);
  eng_->load_state(eng);
  if (h.per_core && (h.per_core != cfg_.per_core || h.clk_base_cyc || h.clk_base_fs)) {
    eng_->set_core_clock(h.per_core, h.clk_base_cyc, h.clk_base_fs);
    cfg_.per_core = h.per_core;
    cfg_.clk_base_cyc = h.clk_base_cyc;
    cfg_.clk_base_fs = h.clk_base_fs;
    cfg_set_divs(cfg_);
    dvfs_ratio_ = (double)per_core_nom_ / (double)h.per_core;
  }
  kernels_done_ = (uint32_t)h.kernels_done;
  tot_cycle_ = h.tot_cycle;
  tot_insn_ = h.tot_insn;
  tot_warp_insn_ = h.tot_warp_insn;
  tot_cta_ = h.tot_cta;
  next_uid_ = (uint32_t)h.next_uid;
  print("GPGPU-Sim: resumed from %s (kernel %u done, cycle %llu)\n", path.c_str(), kernels_done_,
        (unsigned long long)tot_cycle_);
  return (size_t)h.cmd_index + 1;
}

uint64_t Simulator::collective_cycles(const Command& c) const {
  const std::string& m = dopt_.collective_model;
  if (m == "const") return c.coll == "AllReduce" ? (uint64_t)std::max(0, dopt_.nccl_allreduce_latency) : 0;
  // analytic ring / tree model over xGMI (per-link bound: a ring uses one
  // link per direction; the tree uses log2(n) steps)
  const double n = std::max(1, c.nranks);
  if (n <= 1) return 0;
  bool packet_ok = m == "packet";
  if (packet_ok) {
    try {
      coll_kind(c.coll);
    } catch (const std::invalid_argument&) {
      packet_ok = false;  // unknown collective: analytic ring cost below
    }
  }
  if (packet_ok) {
    // standalone run: every rank reaches the collective at the same time and
    // the link model emulates all of them in this process
    CollSpec cs;
    cs.kind = coll_kind(c.coll);
    cs.bytes = c.bytes;
    cs.root = std::max(0, c.root);
    std::vector<uint64_t> start((size_t)c.nranks, 0);
    auto fin = linksim_run_local(link_params(), cs, start);
    uint64_t mx = *std::max_element(fin.begin(), fin.end());
    return (uint64_t)std::ceil((double)mx / core_period_ps());
  }
  const double bw = dopt_.xgmi_link_gbps * 1e9;  // bytes/s per link
  const double alpha = dopt_.xgmi_latency_ns * 1e-9;
  const double S = (double)c.bytes;
  double t = 0;
  const bool tree = m == "tree";
  if (c.coll == "AllReduce") {
    t = tree ? 2 * std::log2(n) * (alpha + S / bw) : 2 * (n - 1) * alpha + 2 * (n - 1) / n * S / bw;
  } else if (c.coll == "AllGather" || c.coll == "ReduceScatter") {
    t = (n - 1) * alpha + (n - 1) / n * S / bw;
  } else if (c.coll == "Broadcast" || c.coll == "Reduce") {
    t = tree ? std::log2(n) * (alpha + S / bw) : (n - 1) * alpha + S / bw;
  } else if (c.coll == "AllToAll") {
    // every GPU exchanges S/n with each peer over its own links
    double links = std::max<uint32_t>(1, dopt_.xgmi_links);
    t = alpha + (n - 1) / n * S / (bw * std::min(links, n - 1));
  } else {
    t = alpha + S / bw;
  }
  const double core_hz = 1e15 / (double)cfg_.per_core;
  return (uint64_t)std::ceil(t * core_hz);
}

LinkParams Simulator::link_params() const {
  LinkParams p;
  p.link_gbps = dopt_.xgmi_link_gbps;
  p.latency_ns = dopt_.xgmi_latency_ns;
  p.links = std::max<uint32_t>(1, dopt_.xgmi_links);
  p.slice_bytes = dopt_.coll_slice_bytes;
  p.max_channels = std::max<uint32_t>(1, dopt_.coll_max_channels);
  p.reduce_gbps = dopt_.coll_reduce_gbps;
  return p;
}

// header, trace and occupancy of a kernel entering the window (reference
// main.cc:94-99 parse_kernel_info + create_kernel_info)
void Simulator::admit_kernel(size_t idx) {
  const Command& c = cmds_[idx];
  std::unique_ptr<StreamOp> op(new StreamOp());
  op->cmd = idx;
  op->t_admit = std::chrono::steady_clock::now();
  op->rk = take_kernel(idx);
  print("Processing kernel %s\n", c.text.c_str());
  setup_kernel_op(*op, true);
  win_.push_back(std::move(op));
}

// occupancy, resources and descriptor of a kernel operation whose ReadyKernel is set
void Simulator::setup_kernel_op(StreamOp& o, bool apply_cta_cap) {
  StreamOp* op = &o;
  if (op->rk->h.warp_size != cfg_.warp_size)
    throw std::runtime_error("trace warp size does not match -gpgpu_shader_core_pipeline");
  const ReadyKernel& rk = *op->rk;
  KernelShape ks{rk.h.block[0] * rk.h.block[1] * rk.h.block[2], rk.h.shmem, rk.h.nregs, rk.n_cta};
  Occupancy occ = compute_occupancy(cfg_, ks);
  if ((uint64_t)occ.cta_per_sm * rk.warps_per_cta > (uint64_t)std::min<uint32_t>(cfg_.max_warps_per_sm, kMaxWarps))
    occ.cta_per_sm = std::max<uint32_t>(1, std::min<uint32_t>(cfg_.max_warps_per_sm, kMaxWarps) / rk.warps_per_cta);
  if (rk.warps_per_cta > (uint32_t)kMaxWarps) throw std::runtime_error("CTA larger than 64 warps");
  KernelDesc& kd = op->kd;
  kd = KernelDesc{};
  kd.uid = next_uid_++;
  kd.n_cta = rk.n_cta;
  kd.stop_when_issued = 0;
  if (apply_cta_cap && dopt_.max_cta > 0) {
    // -gpgpu_max_cta: CTAs past the cap are never issued, and the run ends as
    // soon as the cap is reached (reference gpgpu_sim::active, gpu-sim.cc:1086)
    const uint64_t left = (uint64_t)dopt_.max_cta > tot_cta_ ? (uint64_t)dopt_.max_cta - tot_cta_ : 0;
    if (left <= kd.n_cta) {
      kd.n_cta = (uint32_t)left;
      kd.stop_when_issued = 1;
    }
  }
  kd.warps_per_cta = rk.warps_per_cta;
  kd.threads_per_cta = ks.threads_per_cta;
  kd.shmem_per_cta = rk.h.shmem;
  kd.regs_per_thread = rk.h.nregs;
  kd.cta_per_sm = std::min<uint32_t>(occ.cta_per_sm, kMaxCta);
  for (int i = 0; i < 3; ++i) {
    kd.grid[i] = rk.h.grid[i];
    kd.block[i] = rk.h.block[i];
  }
  kd.stream = (uint32_t)rk.h.stream;
  kd.l1_sets = occ.l1_sets;
  kd.l1_assoc = occ.l1_assoc;
  kd.flush_l1 = (dopt_.flush_l1 ? 1u : 0u) | (dopt_.sqc_invalidate ? 2u : 0u);
  // per-CTA resources for SMs shared by concurrent kernels (the same limits
  // compute_occupancy applies to one kernel)
  const uint32_t padded = (ks.threads_per_cta + cfg_.warp_size - 1) / cfg_.warp_size * cfg_.warp_size;
  kd.thr_cta = padded;
  kd.regs_cta = rk.h.nregs ? padded * ((rk.h.nregs + 3) & ~3u) : 0;
  kd.shmem_cap = occ.shmem_kb ? occ.shmem_kb * 1024u : cfg_.shmem_per_sm;
  kd.shmem_base = rk.h.shmem_base;
  kd.local_base = rk.h.local_base;
  kd.n_insts = rk.insts.size();
  op->occ_limiter = occ.limiter;
  op->stream = rk.h.stream;
  tot_cta_ += kd.n_cta;
}

// -trace_host_budget_mb: a text trace larger than the budget is read per CTA
// as the engine's trace window advances instead of loaded whole
bool Simulator::stream_from_host(const std::string& path) const {
  if (dopt_.host_budget_mb <= 0 || dopt_.engine == "check") return false;
  if (path.size() > 6 && path.compare(path.size() - 6, 6, ".asimk") == 0) return false;
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return false;
  return (double)st.st_size > dopt_.host_budget_mb * 1048576.0;
}

std::unique_ptr<ReadyKernel> Simulator::take_kernel(size_t idx) {
  if (stream_from_host(cmds_[idx].text)) {
    ++host_streamed_;
    return std::unique_ptr<ReadyKernel>(new ReadyKernel(open_streamed_kernel(cmds_[idx].text, cfg_)));
  }
  auto it = pf_.find(idx);
  if (it != pf_.end()) {
    std::unique_ptr<ReadyKernel> k = it->second.get();  // rethrows a loader error
    pf_.erase(it);
    return k;
  }
  return ingest(load_kernel(cmds_[idx].text));
}

std::unique_ptr<ReadyKernel> Simulator::ingest(const HostKernel& k) {
  if (ingest_dev_ < 0 || k.mems.size() < dopt_.gpu_ingest_min) {
    std::unique_ptr<ReadyKernel> r(new ReadyKernel(coalesce_kernel(k, cfg_)));
    if (ingest_dev_ >= 0) {
      std::lock_guard<std::mutex> g(ingest_mu_);
      ++ingest_small_;
    }
    return r;
  }
  IngestStats st;
  std::unique_ptr<ReadyKernel> r(new ReadyKernel(ingest_kernel(k, cfg_, ingest_dev_, &st)));
  std::lock_guard<std::mutex> g(ingest_mu_);
  ingest_st_.smem_jobs += st.smem_jobs;
  ingest_st_.smem_host += st.smem_host;
  ingest_st_.gmem_jobs += st.gmem_jobs;
  ingest_st_.gmem_host += st.gmem_host;
  ingest_st_.mfma += st.mfma;
  ingest_st_.device_s += st.device_s;
  ingest_st_.total_s += st.total_s;
  return r;
}

void Simulator::prefetch_next() {
  if (!dopt_.trace_prefetch || !pf_.empty()) return;
  for (size_t i = next_cmd_; i < cmds_.size(); ++i) {
    if (cmds_[i].type != CMD_KERNEL) continue;
    const std::string path = cmds_[i].text;
    if (stream_from_host(path)) return;  // opened when admitted (reads per CTA)
    pf_[i] = std::async(std::launch::async, [this, path]() { return ingest(load_kernel(path)); });
    return;
  }
}

// start every windowed operation whose stream has no earlier unfinished
// operation (reference main.cc:102-115: busy_streams), kernels in a free
// slot; event records fire at once, event waits end when their record fired
// (repeated until nothing changes: a fired record may release a wait, which
// frees its stream)
void Simulator::launch_ready() {
  for (bool changed = true; changed;) {
    changed = false;
    std::vector<uint64_t> busy;
    for (auto it = win_.begin(); it != win_.end();) {
      StreamOp& op = **it;
      const bool stream_busy = std::find(busy.begin(), busy.end(), op.stream) != busy.end();
      if (op.launched || stream_busy) {
        busy.push_back(op.stream);
        ++it;
        continue;
      }
      if (op.kind == OP_RECORD || (op.kind == OP_WAIT && ev_fired_[op.event] >= op.wait_for)) {
        if (op.kind == OP_RECORD) ev_fired_[op.event]++;
        it = win_.erase(it);
        changed = true;
        continue;
      }
      busy.push_back(op.stream);
      if (op.kind == OP_WAIT) {
        ++it;
        continue;
      }
      if (op.kind == OP_COLL) {
        launch_collective(op);
        changed = true;
        ++it;
        continue;
      }
      int slot = -1;
      for (uint32_t k = 0; k < (uint32_t)std::min<uint32_t>(kMaxConc, (uint32_t)window_size()); ++k)
        if (!slot_op_[k]) {
          slot = (int)k;
          break;
        }
      if (slot < 0) {
        ++it;
        continue;
      }
      if (!eng_->running()) ptrack_.begin_kernel();  // power samples of a busy period
      uint64_t now = eng_->now();
      if (dopt_.host_launch_interval && !dopt_.concurrent_kernel_sm) {
        // host-bound launch: the GPU idles until the host submits the kernel,
        // which then launches into an idle queue; one submitted while the
        // previous kernel still ran is queued behind it
        op.queued = op.submit < now;
        if (op.submit > now && !eng_->running()) {
          eng_->advance(op.submit - now);
          now = eng_->now();
          tot_cycle_ = now;
        }
      }
      const uint64_t lat = (op.queued ? cfg_.kernel_launch_latency_queued : cfg_.kernel_launch_latency) +
                           (op.after_copy ? dopt_.first_kernel_latency : 0);
      op.kd.ready_cycle = now + lat + (uint64_t)cfg_.tb_launch_latency * op.kd.n_cta;
      op.start = now;
      op.start_fs = core_fs(cfg_, now);
      op.slot = slot;
      op.launched = true;
      slot_op_[slot] = &op;
      print("launching kernel name: %s uid: %u\n", op.rk->h.name.c_str(), op.kd.uid);
      print("GPGPU-Sim uArch: CTA/core = %u, limited by: %s\n", op.kd.cta_per_sm, op.occ_limiter);
      eng_->launch((uint32_t)slot, *op.rk, op.kd);
      changed = true;
      ++it;
    }
  }
}

void Simulator::launch_collective(StreamOp& op) {
  const Command& c = cmds_[op.cmd];
  const uint64_t now = eng_->now();
  uint64_t cyc = coll_hook_ ? coll_hook_(c, now) : collective_cycles(c);
  if (c.coll == "AllReduce")
    print("ncclAllReduce was run! Latency: %llu cycles.\n", (unsigned long long)cyc);
  else
    print("%s was run! Latency: %llu cycles.\n", c.text.c_str(), (unsigned long long)cyc);
  op.launched = true;
  op.start = now;
  op.end = now + cyc;
  op.coll_cycles = cyc;
  if (dopt_.coll_mem_traffic) launch_collective_dma(op);
}

// -collective_mem_traffic: the collective's reads of the local send buffer
// and writes of the receive buffer run as an RCCL-style copy kernel in a free
// engine slot (RCCL collectives ARE kernels on the GPU: -collective_max_channels
// workgroups of 256 threads), so they load the simulated L2s, MALL and HBM
// and contend with the compute kernels that overlap them.  The collective
// completes when both the link model's time and the copy kernel are done.
// Per-rank volumes of the ring algorithms: all-reduce 2(n-1)/n x S each way
// (reduce-scatter + all-gather), all-gather / reduce-scatter / all-to-all
// (n-1)/n x S, broadcast / reduce / send-recv S.
void Simulator::launch_collective_dma(StreamOp& op) {
  const Command& c = cmds_[op.cmd];
  const double n = std::max(1, c.nranks);
  if (n <= 1 || c.bytes == 0) return;
  double f = 1.0;
  if (c.coll == "AllReduce") f = 2.0 * (n - 1) / n;
  else if (c.coll == "AllGather" || c.coll == "ReduceScatter" || c.coll == "AllToAll") f = (n - 1) / n;
  const uint64_t bytes = (uint64_t)std::ceil(f * (double)c.bytes);
  int slot = -1;
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
    if (!slot_op_[k]) {
      slot = (int)k;
      break;
    }
  if (slot < 0) {
    print("GPGPU-Sim: WARNING no free kernel slot for the memory traffic of %s: link model only\n", c.text.c_str());
    return;
  }
  const uint64_t now = eng_->now();
  // synthetic buffers: one 4 GiB region per collective command, send half
  // then receive half (the RCCL interposer does not record buffer addresses)
  const uint64_t base = 0x7D0000000000ull + ((uint64_t)op.cmd << 32);
  const uint32_t warps = std::max<uint32_t>(1, 256 / std::max<uint32_t>(1, cfg_.warp_size));
  const uint32_t bv = cfg_.warp_size >= 64 ? 950 : 70;
  std::unique_ptr<StreamOp> d(new StreamOp());
  d->kind = OP_KERNEL;
  d->cmd = op.cmd;
  d->parent = &op;
  d->t_admit = std::chrono::steady_clock::now();
  d->rk.reset(new ReadyKernel(coalesce_kernel(
      make_copy_kernel("rccl_" + c.coll + "_copy", bv, cfg_.warp_size, std::max<uint32_t>(1, dopt_.coll_max_channels),
                       warps, base, bytes, base + (1ull << 31), bytes, op.stream),
      cfg_)));
  setup_kernel_op(*d, false);
  // copy kernels number apart from the trace's kernels (uids stay stable)
  --next_uid_;
  d->kd.uid = 0x40000000u + (uint32_t)(dma_count_++);
  d->kd.ready_cycle = now;  // starts with the collective
  d->start = now;
  d->start_fs = core_fs(cfg_, now);
  d->slot = slot;
  d->launched = true;
  slot_op_[slot] = d.get();
  print("launching kernel name: %s uid: %u (memory traffic of %s, %llu B each way)\n", d->rk->h.name.c_str(),
        d->kd.uid, c.text.c_str(), (unsigned long long)bytes);
  eng_->launch((uint32_t)slot, *d->rk, d->kd);
  op.dma = std::move(d);
  op.dma_pending = true;
}

// advance to the next completion in the window and retire what completed
void Simulator::step() {
  launch_ready();
  prefetch_next();
  uint64_t coll_end = ~0ull;
  for (auto& up : win_)
    if (up->kind == OP_COLL && up->launched && !(up->dma_pending && up->end <= eng_->now()))
      coll_end = std::min(coll_end, up->end);
  if (!eng_->running()) {
    if (coll_end == ~0ull) {
      if (!win_.empty()) throw std::runtime_error("command window stalled: nothing can start");
      return;
    }
    // only collectives in flight: the clock jumps to the first one's end
    const uint64_t now = eng_->now();
    if (coll_end > now) eng_->advance(coll_end - now);
    tot_cycle_ = eng_->now();
    retire_collectives();
    check_limits();
    return;
  }
  RunLimits lim;
  if (dopt_.max_cycle) lim.max_cycle = (uint64_t)dopt_.max_cycle;
  if (coll_end != ~0ull) lim.max_cycle = lim.max_cycle ? std::min(lim.max_cycle, coll_end) : coll_end;
  auto ts = std::chrono::steady_clock::now();
  RunResult rr = (power_ || visualizer_ || cfg_.trace_mask) ? run_sampled(lim) : eng_->run(lim);
  sim_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
  for (auto* op : slot_op_)
    if (op) op->epochs += rr.epochs;
  tot_cycle_ = eng_->now();
  retire_collectives();
  const bool at_max_cycle = (dopt_.max_cycle && eng_->now() >= (uint64_t)dopt_.max_cycle) || dbg_quit_;
  if (rr.cap) cap_hit_ = true;
  if (rr.deadlock) deadlock_ = true;
  // kernels end when they complete, or all together when the run stops
  uint32_t fin = rr.done_mask;
  if (rr.deadlock || rr.cap || at_max_cycle) fin = eng_->running() | rr.done_mask;
  // a queued kernel occupies the command processor at least
  // -sim_kernel_min_cycles_queued (back-to-back dispatch of dependent kernels)
  RunResult rf = rr;
  if (dopt_.kernel_min_cycles_queued && !dopt_.concurrent_kernel_sm && fin == rr.done_mask && !eng_->running()) {
    for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
      if ((fin >> k & 1u) && slot_op_[k] && slot_op_[k]->queued) {
        const uint64_t until = slot_op_[k]->start + (uint64_t)dopt_.kernel_min_cycles_queued;
        if (eng_->now() < until) eng_->advance(until - eng_->now());
      }
    rf.end_cycle = eng_->now();
    tot_cycle_ = eng_->now();
  }
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
    if ((fin >> k & 1u) && slot_op_[k]) finish_kernel(k, rf);
  check_limits();
}

void Simulator::retire_collectives() {
  const uint64_t now = eng_->now();
  for (auto it = win_.begin(); it != win_.end();) {
    StreamOp& op = **it;
    if (op.kind == OP_COLL && op.launched && op.end <= now && !op.dma_pending) {
      const Command& c = cmds_[op.cmd];
      CollectiveResult r;
      r.op = c.coll;
      r.bytes = c.bytes;
      r.nranks = c.nranks;
      r.cycles = op.dma ? std::max<uint64_t>(op.coll_cycles, op.dma_end - op.start) : op.coll_cycles;
      colls_.push_back(r);
      it = win_.erase(it);
    } else {
      ++it;
    }
  }
}

void Simulator::check_limits() {
  if (dbg_quit_) {
    stop_ = true;
    return;
  }
  if (deadlock_) {
    stop_ = true;
    return;
  }
  if (dopt_.max_cycle && (int64_t)tot_cycle_ >= dopt_.max_cycle) {
    print("GPGPU-Sim: ** break due to reaching the maximum cycles (or instructions) **\n");
    stop_ = true;
  } else if ((dopt_.max_insn && (int64_t)tot_insn_ >= dopt_.max_insn) || cap_hit_) {
    print("GPGPU-Sim: ** break due to reaching the maximum cycles (or instructions) **\n");
    stop_ = true;
  }
}

// statistics of a completed kernel (reference main.cc:163-184: print_stats
// when finished_kernel() names it); counters are the deltas since the last
// kernel completed
void Simulator::finish_kernel(uint32_t slot, const RunResult& rr) {
  StreamOp& op = *slot_op_[slot];
  const ReadyKernel& rk = *op.rk;
  const KernelDesc& kd = op.kd;
  // -gpgpu_flush_l2_cache drops the lines (reference l2 flush at kernel
  // end); -sim_l2_kernel_release writes the dirty sectors back first
  if (dopt_.flush_l2 || dopt_.l2_kernel_release) eng_->flush_l2(dopt_.l2_kernel_release);
  std::vector<SMStats> sm;
  std::vector<MemStats> mem;
  eng_->stats(sm, mem);
  if (prev_sm_.empty()) {
    prev_sm_.assign(sm.size(), SMStats{});
    prev_mem_.assign(mem.size(), MemStats{});
  }
  std::vector<SMStats> dsm(sm.size());
  std::vector<MemStats> dmem(mem.size());
  stat_delta(sm, prev_sm_, dsm);
  stat_delta(mem, prev_mem_, dmem);
  prev_sm_ = sm;
  prev_mem_ = mem;
  KernelResult r;
  r.name = rk.h.name;
  r.uid = kd.uid;
  r.start_cycle = op.start;
  r.cycles = rr.end_cycle - op.start;
  r.sim_time_ns = (double)(core_fs(cfg_, rr.end_cycle) - op.start_fs) * 1e-6;
  r.avg_clock_mhz = r.sim_time_ns > 0 ? (double)r.cycles / r.sim_time_ns * 1e3 : 1e9 / (double)per_core_nom_;
  for (auto& s : dsm) {
    r.insn += s.thread_insn;
    r.warp_insn += s.warp_insn;
  }
  r.n_cta = kd.n_cta;
  r.cta_per_sm = kd.cta_per_sm;
  r.ipc = r.cycles ? (double)r.insn / (double)r.cycles : 0;
  {
    double occ_acc = 0, act = 0;
    for (auto& s : dsm) {
      occ_acc += s.occupancy_acc;
      act += s.active_cycles;
    }
    r.occupancy = act > 0 ? 100.0 * occ_acc / (act * cfg_.max_warps_per_sm) : 0;
  }
  r.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - op.t_admit).count();
  r.deadlock = rr.deadlock;
  r.epochs = op.epochs;
  tot_insn_ += r.insn;
  tot_warp_insn_ += r.warp_insn;
  if (power_) {
    r.avg_power_w = ptrack_.kernel_avg_power();
    char hdr[512];
    snprintf(hdr, sizeof(hdr), "kernel_name = %s\nkernel_launch_uid = %u\ngpu_sim_cycle = %llu", r.name.c_str(), r.uid,
             (unsigned long long)r.cycles);
    ptrack_.write_kernel(*power_report_, hdr);
    power_report_->flush();  // the CLI may exit without destroying the simulator
    if (power_steady_) {
      ptrack_.write_steady(*power_steady_, r.name);
      power_steady_->flush();
    }
    if (power_trace_) power_trace_->flush();
    ptrack_.begin_kernel();
  }
  if (visualizer_) visualizer_->flush();
  results_.push_back(r);
  print_kernel_stats(r, dsm, dmem);
  print_sim_time();
  if (rr.deadlock) {
    print("GPGPU-Sim uArch: ERROR ** deadlock detected: last writeback core %u @ gpu_sim_cycle %llu (+ gpu_tot_sim_cycle %llu)\n",
          0u, (unsigned long long)r.cycles, (unsigned long long)op.start);
    // what every stuck unit is waiting for (reference prints the pipeline in
    // debug mode): busy memory channels first, then the SMs
    std::string d = dump_pipeline(-2, -1) + dump_pipeline(-1, -2);
    if (d.size() > 60000) d = d.substr(0, 60000) + "\n... (truncated)\n";
    print("%s", d.c_str());
  }
  // the slot is free again; the operation leaves the window (a collective's
  // copy kernel instead releases its collective)
  slot_op_[slot] = nullptr;
  if (op.parent) {
    op.parent->dma_pending = false;
    op.parent->dma_end = rr.end_cycle;
    return;
  }
  for (auto it = win_.begin(); it != win_.end(); ++it)
    if (it->get() == &op) {
      win_.erase(it);
      break;
    }
  ++kernels_done_;
  if (dopt_.checkpoint_option && kernels_done_ == (uint32_t)dopt_.checkpoint_kernel) ckpt_pending_ = true;
  if (ckpt_pending_ && win_.empty() && !eng_->running()) {
    write_checkpoint(next_cmd_ - 1);
    ckpt_pending_ = false;
  }
}

// Run in gpu_stat_sample_freq slices, one power / visualizer / trace sample
// per slice, until a kernel completes (or a limit stops the run)
RunResult Simulator::run_sampled(const RunLimits& lim0) {
  // HW / HYBRID modes take one sample per kernel (the hardware counters are per kernel)
  const bool hw = power_ && (dopt_.power_mode == 1 || dopt_.power_mode == 2);
  uint64_t freq = std::max<uint64_t>(dopt_.stat_sample_freq, std::max<uint32_t>(1, cfg_.icnt_latency));
  // debugger: one step per slice
  if (dbg_) freq = std::max<uint64_t>(1, dopt_.debug_step ? dopt_.debug_step : cfg_.icnt_latency);
  const double mhz = 1e9 / (double)per_core_nom_;  // nominal: the power model applies the DVFS ratio
  // samples are named after the oldest running kernel
  std::string kname;
  uint32_t best = ~0u;
  for (auto* op : slot_op_)
    if (op && op->kd.uid < best) {
      best = op->kd.uid;
      kname = op->rk->h.name;
    }
  Activity hwa;
  bool have_hw = false;
  if (hw) {
    have_hw = PowerModel::activity_from_hw_csv(dopt_.hw_perf_file, dopt_.hw_perf_bench, kname, hwa, cfg_.n_sm);
    if (!have_hw)
      print("GPGPU-Sim: WARNING no hw_perf entry for bench '%s' kernel '%s' in %s: power uses simulated counters\n",
            dopt_.hw_perf_bench.c_str(), kname.c_str(), dopt_.hw_perf_file.c_str());
  }
  std::vector<SMStats> sm0, sm1, dsm;
  std::vector<MemStats> m0, m1, dm;
  eng_->stats(sm0, m0);
  // power only, at the nominal clock: the engine samples inside its cycle
  // loop (one run, no return to the host per sample); DVFS, HW / HYBRID
  // modes, the visualizer, trace streams and the debugger need the host
  // between samples and run in slices
  if (power_ && !hw && !visualizer_ && !cfg_.trace_mask && !dbg_ && !dopt_.dvfs && dopt_.power_in_loop &&
      eng_->power_sampler()) {
    PwrArm arm;
    arm.coef = power_->sampler_coef(mhz);
    arm.freq = freq;
    arm.t_prev = eng_->now();
    arm.n_sm = cfg_.n_sm;
    {
      std::vector<const SMStats*> sp;
      std::vector<const MemStats*> mp;
      for (auto& x : sm0) sp.push_back(&x);
      for (auto& x : m0) mp.push_back(&x);
      pwr_sums_of(sp.data(), sp.size(), mp.data(), mp.size(), arm.s_prev);
    }
    eng_->power_arm(arm);
    RunResult r;
    try {
      r = eng_->run(lim0);
    } catch (...) {
      eng_->power_disarm();
      throw;
    }
    std::vector<PwrSample> smp;
    eng_->power_drain(smp);
    eng_->power_disarm();
    for (const PwrSample& x : smp) {
      const Activity a = PowerModel::activity_of(x);
      PowerReport p = PowerModel::report_of(x);
      p.clock_ratio = dvfs_ratio_;
      ptrack_.add_sample(p, a, x.now);
      if (power_trace_) ptrack_.write_trace_line(*power_trace_, p, x.now);
    }
    pwr_in_loop_samples_ += smp.size();
    RunResult tot = r;
    tot.hit_limit = r.cap || (lim0.max_cycle && eng_->now() >= lim0.max_cycle);
    return tot;
  }
  RunResult tot;
  uint64_t t_prev = eng_->now();
  for (;;) {
    RunLimits l = lim0;
    if (!hw) {
      const uint64_t nxt = t_prev + freq;
      l.max_cycle = lim0.max_cycle ? std::min<uint64_t>(lim0.max_cycle, nxt) : nxt;
    }
    RunResult r = eng_->run(l);
    tot.epochs += r.epochs;
    tot.end_cycle = r.end_cycle;
    tot.done = r.done;
    tot.done_mask = r.done_mask;
    tot.deadlock = r.deadlock;
    tot.cap = r.cap;
    tot.hit_limit = r.cap;
    const uint64_t now = eng_->now();
    eng_->stats(sm1, m1);
    stat_delta(sm1, sm0, dsm);
    stat_delta(m1, m0, dm);
    if (power_) {
      Activity a = PowerModel::activity_from_stats(dsm, dm, now > t_prev ? now - t_prev : 1);
      if (hw && have_hw) {
        bool use_sim[HW_COUNT];
        for (int i = 0; i < HW_COUNT; ++i) use_sim[i] = dopt_.power_mode == 2 && dopt_.hybrid_use_sim[i];
        a = PowerModel::merge_hw(a, hwa, use_sim);
      }
      PowerReport p = power_->compute(a, mhz, cfg_.n_sm, dvfs_ratio_);
      ptrack_.add_sample(p, a, now);
      if (power_trace_) ptrack_.write_trace_line(*power_trace_, p, now);
      // DVFS governor: the next sample runs at the highest clock whose power,
      // for this sample's per-cycle activity, fits under the measured cap
      if (dopt_.dvfs && !hw) set_clock_ratio(power_->dvfs_clock_ratio(a, mhz, cfg_.n_sm));
    }
    if (visualizer_) write_visualizer_sample(kname, now, now > t_prev ? now - t_prev : 1, dsm, dm);
    if (cfg_.trace_mask) {
      const std::vector<TraceEv> ev = emit_trace();
      if (dbg_ && !dbg_->after_step(now, ev, cfg_.n_sm, (uint32_t)std::min<uint64_t>(cfg_.per_l2, 0xffffffffull),
                                    (uint32_t)std::min<uint64_t>(cfg_.per_core, 0xffffffffull))) {
        dbg_quit_ = true;
        tot.hit_limit = true;
        break;
      }
      if (print_mask_ & TS_LIVENESS) {
        uint64_t insn = 0;
        for (auto& s : dsm) insn += s.thread_insn;
        const double el = std::max(1e-9, wall_seconds());
        print("GPGPU-Sim uArch: cycles simulated: %llu  inst.: %llu (ipc=%4.1f) sim_rate=%llu (inst/sec)\n",
              (unsigned long long)now, (unsigned long long)(tot_insn_ + insn),
              now > t_prev ? (double)insn / (double)(now - t_prev) : 0.0,
              (unsigned long long)((double)(tot_insn_ + insn) / el));
      }
    }
    sm0.swap(sm1);
    m0.swap(m1);
    t_prev = now;
    if (r.done || r.deadlock || r.cap) break;
    if (lim0.max_cycle && now >= lim0.max_cycle) {
      tot.hit_limit = true;
      break;
    }
    if (r.epochs == 0) throw std::runtime_error("power sampling: engine made no progress");
  }
  return tot;
}

// DVFS: from the engine's current cycle on, the core runs at `ratio` x the
// nominal clock.  The time base moves to now, so femtosecond stamps already
// taken (packets in flight, memory-domain ticks) keep their meaning.
void Simulator::set_clock_ratio(double ratio) {
  const uint64_t per = (uint64_t)std::llround((double)per_core_nom_ / ratio);
  if (per == cfg_.per_core) return;
  const uint64_t now = eng_->now();
  const uint64_t base_fs = core_fs(cfg_, now);
  eng_->set_core_clock(per, now, base_fs);
  cfg_.per_core = per;
  cfg_.clk_base_cyc = now;
  cfg_.clk_base_fs = base_fs;
  cfg_set_divs(cfg_);
  dvfs_ratio_ = ratio;
}

// Drain the engine's debug trace buffers and print them DPRINTF-style
// (reference trace.h:56-88: "GPGPU-Sim Cycle N: STREAM - ...") in time order.
std::vector<TraceEv> Simulator::emit_trace() {
  std::vector<TraceEv> ev;
  uint64_t dropped = 0;
  eng_->trace_drain(ev, &dropped);
  auto stream_of = [](uint16_t k) -> uint32_t {
    switch (k) {
      case EV_ISSUE: return TS_WARP_SCHEDULER;
      case EV_SB_RELEASE: return TS_SCOREBOARD;
      case EV_PKT_SEND: case EV_PKT_RECV: return TS_INTERCONNECT;
      case EV_L2_ACCESS: return TS_MEMORY_SUBPARTITION_UNIT;
      case EV_DRAM_CMD: return TS_MEMORY_PARTITION_UNIT;
      default: return 0;
    }
  };
  auto core_time = [&](const TraceEv& e) -> double {
    if (e.kind == EV_L2_ACCESS) return (double)e.cycle * (double)cfg_.per_l2 / (double)cfg_.per_core;
    if (e.kind == EV_DRAM_CMD) return (double)e.cycle * (double)cfg_.per_dram / (double)cfg_.per_core;
    return (double)e.cycle;
  };
  std::vector<size_t> idx(ev.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
    const double ta = core_time(ev[a]), tb = core_time(ev[b]);
    if (ta != tb) return ta < tb;
    return ev[a].unit < ev[b].unit;
  });
  static const char* l2o[] = {"hit", "miss", "mshr-hit", "write-through"};
  static const char* dcmd[] = {"RD", "WR", "ACT", "PRE"};
  for (size_t i : idx) {
    const TraceEv& e = ev[i];
    if (!(print_mask_ & stream_of(e.kind))) continue;  // recorded for the debugger only
    if (dbg_ && e.unit < cfg_.n_sm && print_sm_ >= 0 && e.unit != (uint32_t)print_sm_) continue;
    if (dbg_ && e.unit >= cfg_.n_sm && print_mem_ >= 0 && e.unit - cfg_.n_sm != (uint32_t)print_mem_) continue;
    const unsigned long long cyc = (unsigned long long)core_time(e);
    switch (e.kind) {
      case EV_ISSUE:
        print("GPGPU-Sim Cycle %llu: WARP_SCHEDULER - core %u issued warp %u pc 0x%llx %s\n", cyc, e.unit, e.a,
              (unsigned long long)(e.b & 0xffffffffull), opcode_name((uint16_t)(e.b >> 32)).c_str());
        break;
      case EV_SB_RELEASE:
        print("GPGPU-Sim Cycle %llu: SCOREBOARD - core %u warp %u releases register %llu\n", cyc, e.unit, e.a,
              (unsigned long long)e.b);
        break;
      case EV_PKT_SEND:
        print("GPGPU-Sim Cycle %llu: INTERCONNECT - core %u injects packet to sub-partition %u addr 0x%llx\n", cyc,
              e.unit, e.a, (unsigned long long)e.b);
        break;
      case EV_PKT_RECV:
        print("GPGPU-Sim Cycle %llu: INTERCONNECT - core %u ejects packet type %u addr 0x%llx\n", cyc, e.unit, e.a,
              (unsigned long long)e.b);
        break;
      case EV_L2_ACCESS:
        print("GPGPU-Sim Cycle %llu: MEMORY_SUBPARTITION_UNIT - channel %u sub %u L2 %s line 0x%llx\n", cyc,
              e.unit - cfg_.n_sm, e.a >> 8, l2o[e.a & 3], (unsigned long long)e.b);
        break;
      case EV_DRAM_CMD:
        print("GPGPU-Sim Cycle %llu: MEMORY_PARTITION_UNIT - channel %u DRAM %s bank %llu row %llu\n", cyc,
              e.unit - cfg_.n_sm, dcmd[e.a & 3], (unsigned long long)(e.b >> 32),
              (unsigned long long)(e.b & 0xffffffffull));
        break;
      default: break;
    }
  }
  if (dropped) print("GPGPU-Sim: WARNING %llu trace events dropped (per-unit buffer full)\n", (unsigned long long)dropped);
  return ev;
}

// One line per sample period (reference visualizer_printstat, visualizer.cc:56-84,
// whose gz log feeds AerialVision): global counters plus per-SM instruction
// counts, so activity over time can be plotted per core.
void Simulator::write_visualizer_sample(const std::string& kname, uint64_t now, uint64_t cycles,
                                        const std::vector<SMStats>& dsm, const std::vector<MemStats>& dm) {
  uint64_t insn = 0, l1_acc = 0, l1_miss = 0, l2_acc = 0, l2_miss = 0, drd = 0, dwr = 0, busy = 0, dcyc = 0;
  for (auto& s : dsm) {
    insn += s.thread_insn;
    for (int t = 0; t < L1T_COUNT; ++t) {
      for (int o = 0; o < L1O_COUNT; ++o) l1_acc += s.l1[t][o];
      l1_miss += s.l1[t][L1O_MISS];
    }
  }
  for (auto& m : dm) {
    for (int t = 0; t < L2T_COUNT; ++t) {
      l2_acc += m.l2[t][L2O_HIT] + m.l2[t][L2O_MISS] + m.l2[t][L2O_MSHR_HIT];
      l2_miss += m.l2[t][L2O_MISS];
    }
    drd += m.dram_rd;
    dwr += m.dram_wr;
    busy += m.dram_busy_cycles;
    dcyc += m.dram_cycles;
  }
  std::ostream& o = *visualizer_;
  o << "kernel=" << kname << " cycle=" << now << " period=" << cycles << " insn=" << insn
    << " ipc=" << (double)insn / (double)cycles << " l1_access=" << l1_acc << " l1_miss=" << l1_miss
    << " l2_access=" << l2_acc << " l2_miss=" << l2_miss << " dram_rd=" << drd << " dram_wr=" << dwr
    << " dram_util=" << (dcyc ? (double)busy / (double)dcyc : 0.0) << " sm_insn=";
  for (size_t i = 0; i < dsm.size(); ++i) o << (i ? "," : "") << dsm[i].warp_insn;
  // per-unit vectors (reference: per-shader L1 miss rates, visualizer.cc:84-110;
  // per-DRAM-channel dramutil / drameff / dramnreq, dram.cc:815-853; per
  // sub-partition L2 hits and misses, l2cache.cc:866)
  auto vec = [&](const char* key, size_t n, auto f) {
    o << " " << key << "=";
    for (size_t i = 0; i < n; ++i) o << (i ? "," : "") << f(i);
  };
  auto l1_miss_rate = [&](size_t i) {
    uint64_t a = 0, m = 0;
    for (int t = 0; t < L1T_COUNT; ++t) {
      for (int oo = 0; oo < L1O_COUNT; ++oo) a += dsm[i].l1[t][oo];
      m += dsm[i].l1[t][L1O_MISS];
    }
    return a ? (double)m / (double)a : 0.0;
  };
  vec("sm_l1_miss_rate", dsm.size(), l1_miss_rate);
  vec("sm_occupancy", dsm.size(), [&](size_t i) { return (double)dsm[i].occupancy_acc / (double)cycles; });
  vec("sm_active", dsm.size(), [&](size_t i) { return (double)dsm[i].active_cycles / (double)cycles; });
  vec("sm_pkts_out", dsm.size(), [&](size_t i) { return dsm[i].pkts_out; });
  // global issue distribution: idle, scoreboard, stall, then issued with k
  // active lanes (the warp-divergence breakdown AerialVision stacks)
  vec("issue_distro", 3 + (size_t)kMaxWarpLanes, [&](size_t k) {
    uint64_t v = 0;
    for (auto& s : dsm) v += s.issue_distro[k];
    return v;
  });
  vec("mf_lat_hist", 16, [&](size_t k) {
    uint64_t v = 0;
    for (auto& s : dsm) v += s.mf_lat_hist[k];
    return v;
  });
  {
    uint64_t n = 0, sum = 0;
    for (auto& s : dsm) {
      n += s.mf_lat_n;
      sum += s.mf_lat_sum;
    }
    o << " mf_lat_avg=" << (n ? (double)sum / (double)n : 0.0);
  }
  vec("ch_dram_util", dm.size(),
      [&](size_t i) { return dm[i].dram_cycles ? (double)dm[i].dram_busy_cycles / (double)dm[i].dram_cycles : 0.0; });
  // mean requests queued at the channel (reference dramavemrqs)
  vec("ch_dram_queue", dm.size(),
      [&](size_t i) { return dm[i].dram_cycles ? (double)dm[i].dram_q_occ / (double)dm[i].dram_cycles : 0.0; });
  vec("ch_dram_req", dm.size(), [&](size_t i) { return dm[i].dram_rd + dm[i].dram_wr; });
  vec("ch_dram_act", dm.size(), [&](size_t i) { return dm[i].dram_act; });
  vec("ch_l2_hit", dm.size(), [&](size_t i) {
    uint64_t v = 0;
    for (int t = 0; t < L2T_COUNT; ++t) v += dm[i].l2[t][L2O_HIT];
    return v;
  });
  vec("ch_l2_miss", dm.size(), [&](size_t i) {
    uint64_t v = 0;
    for (int t = 0; t < L2T_COUNT; ++t) v += dm[i].l2[t][L2O_MISS];
    return v;
  });
  o << "\n";
}

void Simulator::print_kernel_stats(const KernelResult& r, const std::vector<SMStats>& sm,
                                   const std::vector<MemStats>& mem) {
  print("kernel_name = %s \n", r.name.c_str());
  print("kernel_launch_uid = %u \n", r.uid);
  print("gpu_sim_cycle = %llu\n", (unsigned long long)r.cycles);
  print("gpu_sim_insn = %llu\n", (unsigned long long)r.insn);
  print("gpu_ipc = %12.4f\n", r.ipc);
  if (dopt_.dvfs) {
    // DVFS: the core clock followed the power cap, so cycles != time
    print("gpu_sim_time_ns = %.1f\n", r.sim_time_ns);
    print("gpu_avg_core_clock_mhz = %.1f\n", r.avg_clock_mhz);
  }
  print("gpu_tot_sim_cycle = %llu\n", (unsigned long long)tot_cycle_);
  print("gpu_tot_sim_insn = %llu\n", (unsigned long long)tot_insn_);
  print("gpu_tot_ipc = %12.4f\n", tot_cycle_ ? (double)tot_insn_ / (double)tot_cycle_ : 0.0);
  print("gpu_tot_issued_cta = %llu\n", (unsigned long long)tot_cta_);
  print("gpu_occupancy = %.4f%% \n", r.occupancy);
  print("gpu_tot_occupancy = %.4f%% \n", r.occupancy);
  {
    // this kernel's mean L1-miss round trip (MSHR allocation -> last sector), core cycles
    uint64_t n = 0, sum = 0;
    for (auto& st : sm) {
      n += st.mf_lat_n;
      sum += st.mf_lat_sum;
    }
    print("L1_miss_avg_latency = %.2f\n", n ? (double)sum / (double)n : 0.0);
  }
  uint64_t l2_bytes = 0, dram_rd = 0, dram_wr = 0, dram_act = 0, dram_busy = 0, dram_cyc = 0;
  uint64_t l2[L2T_COUNT][L2O_COUNT] = {};
  // Rates (bandwidths, utilisation) are this kernel's; event counts are
  // cumulative over the run like the reference's (gpu-sim.cc:1355-1541 print
  // the never-reset shader / cache / DRAM counters; get_stats.py differences
  // them per kernel as collect_aggregate).
  const std::vector<SMStats>& csm = prev_sm_;
  const std::vector<MemStats>& cmem = prev_mem_;
  for (auto& m : mem) {
    l2_bytes += m.bytes_in + m.bytes_out;
    dram_busy += m.dram_busy_cycles;
    dram_cyc += m.dram_cycles;
  }
  for (auto& m : cmem) {
    dram_rd += m.dram_rd;
    dram_wr += m.dram_wr;
    dram_act += m.dram_act;
    for (int t = 0; t < L2T_COUNT; ++t)
      for (int o = 0; o < L2O_COUNT; ++o) l2[t][o] += m.l2[t][o];
  }
  const double secs = r.cycles * (double)cfg_.per_core * 1e-15;
  print("L2_BW  = %12.4f GB/Sec\n", secs > 0 ? l2_bytes / secs / 1e9 : 0.0);
  print("L2_BW_total  = %12.4f GB/Sec\n", secs > 0 ? l2_bytes / secs / 1e9 : 0.0);
  print("gpu_total_sim_rate=%llu\n", (unsigned long long)(tot_insn_ / std::max(1e-9, sim_s_)));
  // L1 breakdown (names follow the reference's mem_access_type / cache
  // request status strings so get_stats.py regexes keep working)
  static const char* l1t[L1T_COUNT] = {"GLOBAL_ACC_R", "GLOBAL_ACC_W", "LOCAL_ACC_R", "LOCAL_ACC_W", "GLOBAL_ATOMIC"};
  uint64_t l1[L1T_COUNT][L1O_COUNT] = {};
  uint64_t shm = 0, shm_conf = 0, lk64 = 0;
  for (auto& s : csm) {
    lk64 += s.l1_lookups64;
    for (int t = 0; t < L1T_COUNT; ++t)
      for (int o = 0; o < L1O_COUNT; ++o) l1[t][o] += s.l1[t][o];
    shm += s.shmem_acc;
    shm_conf += s.shmem_conflict_cycles;
  }
  print("\nTotal_core_cache_stats:\n");
  for (int t = 0; t < L1T_COUNT; ++t) {
    uint64_t tot = 0;
    for (int o = 0; o < L1O_COUNT; ++o)
      if (o != L1O_RES_FAIL) tot += l1[t][o];
    print("\tTotal_core_cache_stats_breakdown[%s][HIT] = %llu\n", l1t[t], (unsigned long long)l1[t][L1O_HIT]);
    print("\tTotal_core_cache_stats_breakdown[%s][MISS] = %llu\n", l1t[t],
          (unsigned long long)(l1[t][L1O_MISS] + l1[t][L1O_BYPASS]));
    print("\tTotal_core_cache_stats_breakdown[%s][MSHR_HIT] = %llu\n", l1t[t], (unsigned long long)l1[t][L1O_MSHR_HIT]);
    print("\tTotal_core_cache_stats_breakdown[%s][TOTAL_ACCESS] = %llu\n", l1t[t], (unsigned long long)tot);
  }
  print("\tL1D_total_64B_tag_lookups = %llu\n", (unsigned long long)lk64);
  print("\nTotal_core_cache_fail_stats:\n");
  for (int t = 0; t < L1T_COUNT; ++t)
    print("\tTotal_core_cache_fail_stats_breakdown[%s][MSHR_ENRTY_FAIL] = %llu\n", l1t[t],
          (unsigned long long)l1[t][L1O_RES_FAIL]);
  {
    // instruction cache, cumulative over the run (reference shader.cc:3051-3074)
    uint64_t ic[4] = {};
    for (auto& st : prev_sm_)
      for (int i = 0; i < 4; ++i) ic[i] += st.il1[i];
    const uint64_t acc = ic[IL1_HIT] + ic[IL1_MISS] + ic[IL1_MSHR_HIT];
    print("\tL1I_total_cache_accesses = %llu\n", (unsigned long long)acc);
    print("\tL1I_total_cache_misses = %llu\n", (unsigned long long)ic[IL1_MISS]);
    if (acc) print("\tL1I_total_cache_miss_rate = %.4lf\n", (double)ic[IL1_MISS] / (double)acc);
    print("\tL1I_total_cache_pending_hits = %llu\n", (unsigned long long)ic[IL1_MSHR_HIT]);
    print("\tL1I_total_cache_reservation_fails = %llu\n", (unsigned long long)ic[IL1_RES_FAIL]);
    uint64_t pf = 0;
    for (auto& st : prev_sm_) pf += st.il1_prefetch;
    if (cfg_.inst_prefetch) print("\tL1I_total_cache_prefetches = %llu\n", (unsigned long long)pf);
  }
  print("gpgpu_n_shmem_bank_access = %llu\n", (unsigned long long)shm);
  print("gpgpu_n_shmem_bkconflict = %llu\n", (unsigned long long)shm_conf);
  static const char* l2t[L2T_COUNT] = {"GLOBAL_ACC_R", "GLOBAL_ACC_W", "GLOBAL_ATOMIC"};
  print("\nL2_cache_stats:\n");
  for (int t = 0; t < L2T_COUNT; ++t) {
    uint64_t tot = l2[t][L2O_HIT] + l2[t][L2O_MISS] + l2[t][L2O_MSHR_HIT];
    print("\tL2_cache_stats_breakdown[%s][HIT] = %llu\n", l2t[t], (unsigned long long)l2[t][L2O_HIT]);
    print("\tL2_cache_stats_breakdown[%s][MISS] = %llu\n", l2t[t], (unsigned long long)l2[t][L2O_MISS]);
    print("\tL2_cache_stats_breakdown[%s][MSHR_HIT] = %llu\n", l2t[t], (unsigned long long)l2[t][L2O_MSHR_HIT]);
    print("\tL2_cache_stats_breakdown[%s][TOTAL_ACCESS] = %llu\n", l2t[t], (unsigned long long)tot);
  }
  uint64_t l2_tot = 0, l2_miss = 0;
  for (int t = 0; t < L2T_COUNT; ++t) {
    l2_tot += l2[t][L2O_HIT] + l2[t][L2O_MISS] + l2[t][L2O_MSHR_HIT];
    l2_miss += l2[t][L2O_MISS];
  }
  print("L2_total_cache_accesses = %llu\n", (unsigned long long)l2_tot);
  print("L2_total_cache_misses = %llu\n", (unsigned long long)l2_miss);
  print("L2_total_cache_miss_rate = %.4f\n", l2_tot ? (double)l2_miss / l2_tot : 0.0);
  print("total dram reads = %llu\n", (unsigned long long)dram_rd);
  print("total dram writes = %llu\n", (unsigned long long)dram_wr);
  print("total dram activates = %llu\n", (unsigned long long)dram_act);
  {
    // traffic leaving the L2 for memory (Infinity Fabric on CDNA4: what
    // rocprofv3 counts as TCC_EA0_RDREQ / WRREQ) and the MALL in front of DRAM
    uint64_t mrd = 0, mwr = 0, mh = 0, mm = 0, mw = 0, mwb = 0, mrq = 0, mwq = 0;
    for (auto& m : cmem) {
      mrd += m.l2_mem_rd;
      mwr += m.l2_mem_wr;
      mrq += m.l2_mem_rd_req;
      mwq += m.l2_mem_wr_req;
      mh += m.mall_rd_hit;
      mm += m.mall_rd_miss;
      mw += m.mall_wr;
      mwb += m.mall_wb;
    }
    print("L2_to_mem_read_sectors = %llu\n", (unsigned long long)mrd);
    print("L2_to_mem_write_sectors = %llu\n", (unsigned long long)mwr);
    print("L2_to_mem_read_requests = %llu\n", (unsigned long long)mrq);
    print("L2_to_mem_write_requests = %llu\n", (unsigned long long)mwq);
    if (cfg_.mall_sets) {
      print("MALL_read_hits = %llu\n", (unsigned long long)mh);
      print("MALL_read_misses = %llu\n", (unsigned long long)mm);
      print("MALL_read_hit_rate = %.4f\n", mh + mm ? (double)mh / (double)(mh + mm) : 0.0);
      print("MALL_writes = %llu\n", (unsigned long long)mw);
      print("MALL_writebacks = %llu\n", (unsigned long long)mwb);
    }
    if (cfg_.n_xcd) print("XCDs = %u (private L2 slices per XCD = %u)\n", cfg_.n_xcd, 1u << cfg_.log2_spx);
  }
  print("dram_bw_util = %.4f\n", dram_cyc ? (double)dram_busy / dram_cyc : 0.0);
  {
    // per memory channel and per L2 bank (reference dram_t::print and the
    // L2_cache_bank lines of gpgpu_sim::print_stats, cumulative counters;
    // utilisation over this kernel)
    const uint32_t per = std::max<uint32_t>(1, cfg_.n_sub_per_mem);
    uint64_t icnt_stall = 0, dram_full = 0;
    for (size_t ch = 0; ch * per < cmem.size(); ++ch) {
      uint64_t rd = 0, wr = 0, act = 0, pre = 0, busy = 0, cyc = 0;
      for (uint32_t j = 0; j < per && ch * per + j < cmem.size(); ++j) {
        const MemStats& m = cmem[ch * per + j];
        rd += m.dram_rd;
        wr += m.dram_wr;
        act += m.dram_act;
        pre += m.dram_pre;
        if (ch * per + j < mem.size()) {
          busy += mem[ch * per + j].dram_busy_cycles;
          cyc += mem[ch * per + j].dram_cycles;
        }
      }
      print("DRAM[%zu]: n_act=%llu n_pre=%llu n_rd=%llu n_write=%llu bw_util=%.4f\n", ch, (unsigned long long)act,
            (unsigned long long)pre, (unsigned long long)rd, (unsigned long long)wr, cyc ? (double)busy / cyc : 0.0);
    }
    for (size_t b = 0; b < cmem.size(); ++b) {
      const MemStats& m = cmem[b];
      uint64_t acc = 0, miss = 0;
      for (int t = 0; t < L2T_COUNT; ++t) {
        acc += m.l2[t][L2O_HIT] + m.l2[t][L2O_MISS] + m.l2[t][L2O_MSHR_HIT];
        miss += m.l2[t][L2O_MISS];
      }
      print("L2_cache_bank[%zu]: Access = %llu, Miss = %llu, Miss_rate = %.3f, Pending_hits = %llu, Reservation_fails = %llu\n",
            b, (unsigned long long)acc, (unsigned long long)miss, acc ? (double)miss / acc : 0.0,
            (unsigned long long)(m.l2[L2T_RD][L2O_MSHR_HIT] + m.l2[L2T_WR][L2O_MSHR_HIT] + m.l2[L2T_ATOM][L2O_MSHR_HIT]),
            (unsigned long long)(m.l2[L2T_RD][L2O_RES_FAIL] + m.l2[L2T_WR][L2O_RES_FAIL] + m.l2[L2T_ATOM][L2O_RES_FAIL]));
      icnt_stall += m.icnt_stall;
      dram_full += m.l2[L2T_RD][L2O_RES_FAIL] + m.l2[L2T_WR][L2O_RES_FAIL] + m.l2[L2T_ATOM][L2O_RES_FAIL];
    }
    print("gpu_stall_dramfull = %llu\n", (unsigned long long)dram_full);
    print("gpu_stall_icnt2sh    = %llu\n", (unsigned long long)icnt_stall);
  }
  print("gpgpu_n_tot_w_icount = %llu\n", (unsigned long long)tot_warp_insn_);
  {
    // crossbar subnets (reference LocalInterconnect::DisplayStats,
    // local_interconnect.cc:360-420): request net = SM -> L2 ports, reply
    // net = L2 -> SM ports; conflicts = ready inputs a port did not grant
    uint64_t rq_pk = 0, rq_cf = 0, rq_ac = 0, rq_q = 0, rp_pk = 0, rp_cf = 0, rp_q = 0;
    for (auto& m : cmem) {
      rq_pk += m.pkts_in;
      rq_cf += m.icnt_conflicts;
      rq_ac += m.icnt_arb_cycles;
      rq_q += m.icnt_queue_cycles;
    }
    for (auto& st : csm) {
      rp_pk += st.pkts_in;
      rp_cf += st.icnt_reply_conflicts;
      rp_q += st.icnt_reply_queue_cycles;
    }
    print("Req_Network_injected_packets_num = %llu\n", (unsigned long long)rq_pk);
    print("Req_Network_conflicts = %llu\n", (unsigned long long)rq_cf);
    print("Req_Network_conflicts_per_cycle_util = %.4f\n", rq_ac ? (double)rq_cf / (double)rq_ac : 0.0);
    print("Req_Network_queueing_cycles = %llu\n", (unsigned long long)rq_q);
    print("Req_Network_avg_queueing_cycles = %.4f\n", rq_pk ? (double)rq_q / (double)rq_pk : 0.0);
    print("Reply_Network_injected_packets_num = %llu\n", (unsigned long long)rp_pk);
    print("Reply_Network_conflicts = %llu\n", (unsigned long long)rp_cf);
    print("Reply_Network_queueing_cycles = %llu\n", (unsigned long long)rp_q);
    print("Reply_Network_avg_queueing_cycles = %.4f\n", rp_pk ? (double)rp_q / (double)rp_pk : 0.0);
    if (icnt_contention_on(cfg_)) {
      // cumulative over the run: packets a busy link delayed, and the delay
      uint64_t dl = 0, wc = 0, dd = 0;
      eng_->link_stats(&dl, &wc, &dd);
      print("Network_link_delayed_packets = %llu\n", (unsigned long long)dl);
      print("Network_link_wait_cycles = %llu\n", (unsigned long long)wc);
      if (cfg_.link_contention == 2) {
        // injection back-pressure (HasBuffer): cycles a ready packet waited
        // for room in its node's injection queue, SM side and L2 side
        uint64_t sm_inj = 0, l2_inj = 0;
        for (auto& st : csm) sm_inj += st.icnt_inj_stall;
        for (auto& m : cmem) l2_inj += m.icnt_inj_stall;
        print("Req_Network_injection_stall_cycles = %llu\n", (unsigned long long)sm_inj);
        print("Reply_Network_injection_stall_cycles = %llu\n", (unsigned long long)l2_inj);
        print("Network_router_deadlocked_packets = %llu\n", (unsigned long long)dd);
        if (dd) print("GPGPU-Sim: WARNING: %llu packets met a routing deadlock in the router model; they kept their "
                      "uncontended latency\n", (unsigned long long)dd);
      }
    }
  }
  {
    // further gpu_print_stat / shader_core_stats lines (reference
    // gpu-sim.cc:1355-1541, shader.cc:3012-3170): instruction mix, issue
    // stalls, register-bank conflicts, dual issue, L1 write-backs; memory
    // partition, DRAM queue and interconnect stalls
    uint64_t cls[OC_COUNT] = {}, stall_idle = 0, sb = 0, pipe = 0, bankc = 0, dual = 0, l1wb = 0, l1wbl = 0,
             act = 0, busyc = 0, occ = 0, rfr = 0, rfw = 0, ctas = 0, warps = 0, memi = 0;
    for (auto& st : csm) {
      for (int i = 0; i < OC_COUNT; ++i) cls[i] += st.cls_insn[i];
      stall_idle += st.issue_stall_idle;
      sb += st.sb_stall;
      pipe += st.pipe_stall;
      bankc += st.oc_bank_conflicts;
      dual += st.dual_issued;
      l1wb += st.l1_wb;
      l1wbl += st.l1_wb_lost;
      act += st.active_cycles;
      busyc += st.busy_cycles;
      occ += st.occupancy_acc;
      rfr += st.rf_reads;
      rfw += st.rf_writes;
      ctas += st.ctas_done;
      warps += st.warps_done;
      memi += st.mem_insn;
    }
    print("gpgpu_n_load_insn = %llu\n", (unsigned long long)cls[OC_LOAD]);
    print("gpgpu_n_store_insn = %llu\n", (unsigned long long)cls[OC_STORE]);
    print("gpgpu_n_mem_insn_dispatched = %llu\n", (unsigned long long)memi);
    print("gpgpu_n_branch_insn = %llu\n", (unsigned long long)cls[OC_BRANCH]);
    print("gpgpu_n_sfu_insn = %llu\n", (unsigned long long)cls[OC_SFU]);
    print("gpgpu_n_dp_insn = %llu\n", (unsigned long long)cls[OC_DP]);
    print("gpgpu_n_tensor_insn = %llu\n", (unsigned long long)cls[OC_TENSOR]);
    print("gpgpu_n_barrier_insn = %llu\n", (unsigned long long)cls[OC_BARRIER]);
    {
      // wave instructions by the CDNA sequencer counter classes (SQ_INSTS_*)
      uint64_t sq[8] = {};
      for (auto& st : csm)
        for (int i = 0; i < 8; ++i) sq[i] += st.sq_insn[i];
      static const char* sqn[8] = {"valu", "salu", "smem", "vmem_rd", "vmem_wr", "lds", "sq_branch", "other"};
      for (int i = 0; i < 8; ++i) print("gpgpu_n_%s_insn = %llu\n", sqn[i], (unsigned long long)sq[i]);
    }
    print("gpgpu_n_dual_issue = %llu\n", (unsigned long long)dual);
    {
      // reference shader_core_stats::print (shader.cc:724-740), cumulative
      uint64_t dist[3 + kMaxWarpLanes] = {}, si[kMaxSched] = {}, di[kMaxSched] = {};
      for (auto& st : csm) {
        for (int i = 0; i < 3 + kMaxWarpLanes; ++i) dist[i] += st.issue_distro[i];
        for (int i = 0; i < kMaxSched; ++i) {
          si[i] += st.single_issue[i];
          di[i] += st.dual_issue[i];
        }
      }
      std::string l = "Stall:" + std::to_string(dist[2]) + "\tW0_Idle:" + std::to_string(dist[0]) +
                      "\tW0_Scoreboard:" + std::to_string(dist[1]);
      const uint32_t ws = std::min<uint32_t>(cfg_.warp_size, kMaxWarpLanes);
      for (uint32_t i = 1; i <= ws; ++i) l += "\tW" + std::to_string(i) + ":" + std::to_string(dist[2 + i]);
      print("Warp Occupancy Distribution:\n%s\n", l.c_str());
      std::string a = "single_issue_nums: ", b = "dual_issue_nums: ";
      const uint32_t ns = std::max<uint32_t>(1, std::min<uint32_t>(cfg_.n_sched, kMaxSched));
      for (uint32_t i = 0; i < ns; ++i) {
        a += "WS" + std::to_string(i) + ":" + std::to_string(si[i]) + "\t";
        b += "WS" + std::to_string(i) + ":" + std::to_string(di[i]) + "\t";
      }
      print("%s\n%s\n", a.c_str(), b.c_str());
    }
    print("gpu_stall_shd_idle_sched = %llu\n", (unsigned long long)stall_idle);
    print("gpgpu_n_stall_shd_mem = %llu\n",
          (unsigned long long)(l1[L1T_GLOBAL_R][L1O_RES_FAIL] + l1[L1T_GLOBAL_W][L1O_RES_FAIL] +
                               l1[L1T_LOCAL_R][L1O_RES_FAIL] + l1[L1T_LOCAL_W][L1O_RES_FAIL] +
                               l1[L1T_ATOMIC][L1O_RES_FAIL]));
    print("gpu_stall_result_bus = %llu\n", (unsigned long long)pipe);
    print("gpu_reg_bank_conflict_stalls = %llu\n", (unsigned long long)bankc);
    print("gpgpu_n_l1_writebacks = %llu\n", (unsigned long long)l1wb);
    if (l1wbl) print("GPGPU-Sim uArch: WARNING ** %llu L1 write-backs lost to a full injection queue\n",
                     (unsigned long long)l1wbl);
    print("gpgpu_n_regfile_reads = %llu\n", (unsigned long long)rfr);
    print("gpgpu_n_regfile_writes = %llu\n", (unsigned long long)rfw);
    print("gpgpu_n_completed_cta = %llu\n", (unsigned long long)ctas);
    print("gpgpu_n_completed_warps = %llu\n", (unsigned long long)warps);
    print("gpgpu_sm_active_cycles = %llu\n", (unsigned long long)act);
    print("gpgpu_sm_issue_busy_cycles = %llu\n", (unsigned long long)busyc);
    print("gpgpu_avg_active_warps = %.4f\n", act ? (double)occ / (double)act : 0.0);
    uint64_t l2cyc = 0, l2busy = 0, rop = 0, qocc = 0, icst = 0, pre = 0, evd = 0, cdc = 0;
    for (auto& m : cmem) {
      cdc += m.dram_cycles;
      l2cyc += m.l2_cycles;
      l2busy += m.l2_busy;
      rop += m.rop_occ;
      qocc += m.dram_q_occ;
      icst += m.icnt_stall;
      pre += m.dram_pre;
      evd += m.l2_evict_dirty;
    }
    (void)icst;  // gpu_stall_dramfull / gpu_stall_icnt2sh are printed once, with the L2 bank lines
    print("L2_cache_dirty_evictions = %llu\n", (unsigned long long)evd);
    print("L2_busy_rate = %.4f\n", l2cyc ? (double)l2busy / (double)l2cyc : 0.0);
    print("avg_rop_queue_occupancy = %.4f\n", l2cyc ? (double)rop / (double)l2cyc : 0.0);
    print("avg_dram_sched_queue_occupancy = %.4f\n", cdc ? (double)qocc / (double)cdc : 0.0);
    print("total dram precharges = %llu\n", (unsigned long long)pre);
    print("dram_row_buffer_locality = %.4f\n",
          (dram_rd + dram_wr) ? 1.0 - (double)dram_act / (double)(dram_rd + dram_wr) : 0.0);
  }
  uint64_t pk_out = 0, pk_in = 0;
  for (auto& s : csm) {
    pk_out += s.pkts_out;
    pk_in += s.pkts_in;
  }
  {
    uint64_t bl = 0, drop = 0;
    for (auto& m : cmem) {
      bl += m.icnt_backlog;
      drop += m.icnt_ovf_drop;
    }
    print("icnt_mem_input_backlog = %llu\n", (unsigned long long)bl);
    if (drop) print("GPGPU-Sim uArch: WARNING ** %llu interconnect packets lost to a full backlog ring\n",
                    (unsigned long long)drop);
  }
  print("icnt_total_pkts_mem_to_simt = %llu\n", (unsigned long long)pk_in);
  print("icnt_total_pkts_simt_to_mem = %llu\n", (unsigned long long)pk_out);
  if (dopt_.memlatency_stat) {
    // L1 miss round trips, cumulative over the run like the reference's
    // memory_stats_t::memlatstat_print (prev_sm_ holds the raw counters here)
    uint64_t n = 0, sum = 0, mx = 0, hist[16] = {};
    for (auto& s : prev_sm_) {
      n += s.mf_lat_n;
      sum += s.mf_lat_sum;
      mx = std::max<uint64_t>(mx, s.mf_lat_max);
      for (int i = 0; i < 16; ++i) hist[i] += s.mf_lat_hist[i];
    }
    print("maxmflatency = %llu \n", (unsigned long long)mx);
    print("averagemflatency = %llu \n", (unsigned long long)(n ? sum / n : 0));
    print("mf_lat_table:");
    for (int i = 0; i < 16; ++i) print("%llu \t", (unsigned long long)hist[i]);
    print("\n");
  }
  if (power_) print("gpu_avg_power = %.4f W\n", r.avg_power_w);
}

void Simulator::print_sim_time() {
  double el = wall_seconds();
  unsigned long long d = (unsigned long long)std::max(1.0, std::ceil(el));
  unsigned long long dd = d / 86400, hh = d / 3600 % 24, mm = d / 60 % 60, ss = d % 60;
  print("\n\ngpgpu_simulation_time = %llu days, %llu hrs, %llu min, %llu sec (%llu sec)\n", dd, hh, mm, ss, d);
  double rate_s = std::max(1e-9, el);
  print("gpgpu_simulation_rate = %llu (inst/sec)\n", (unsigned long long)(tot_insn_ / rate_s));
  unsigned long long cps = (unsigned long long)(tot_cycle_ / rate_s);
  print("gpgpu_simulation_rate = %llu (cycle/sec)\n", cps);
  double core_khz = 1e12 / (double)cfg_.per_core;
  print("gpgpu_silicon_slowdown = %llux\n", cps ? (unsigned long long)(core_khz * 1000.0 / cps) : 0ull);
  uint64_t peak = 0, refills = 0;
  eng_->trace_residency(&peak, &refills);
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
    if (slot_op_[k] && slot_op_[k]->rk && slot_op_[k]->rk->streamed())
      host_stream_peak_ = std::max(host_stream_peak_, slot_op_[k]->rk->host_peak_bytes);
  if (pwr_in_loop_samples_) print("power_in_loop_samples: %llu\n", (unsigned long long)pwr_in_loop_samples_);
  if (eng_->launches()) print("engine_kernel_launches: %llu\n", (unsigned long long)eng_->launches());
  if (host_streamed_)
    print("trace_host_streamed_kernels: %llu\ntrace_host_peak_bytes: %llu\n", (unsigned long long)host_streamed_,
          (unsigned long long)host_stream_peak_);
  // not "key = value": an engine diagnostic, not a statistic of the model
  if (peak)
    print("gpu_trace_resident_peak_bytes: %llu\ngpu_trace_window_fills: %llu\n", (unsigned long long)peak,
          (unsigned long long)refills);
  if (ingest_dev_ >= 0) {
    std::lock_guard<std::mutex> g(ingest_mu_);
    print("gpu_ingest: shared %llu on device (%llu host), global %llu on device (%llu host), %llu mfma, "
          "device %.3f s of %.3f s, %llu small kernels on the host\n",
          (unsigned long long)ingest_st_.smem_jobs, (unsigned long long)ingest_st_.smem_host,
          (unsigned long long)ingest_st_.gmem_jobs, (unsigned long long)ingest_st_.gmem_host,
          (unsigned long long)ingest_st_.mfma, ingest_st_.device_s, ingest_st_.total_s,
          (unsigned long long)ingest_small_);
  }
  fflush(stdout);
}

}  // namespace asim
