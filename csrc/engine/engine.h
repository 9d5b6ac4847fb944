// Cycle-engine interface.  Two implementations run the SAME model code
// (csrc/model): the CPU reference engine (cpu_engine.cc, SeqPar) and the
// MI355X engine (gpu_engine.hip, one wavefront per SM / memory channel,
// persistent kernel with one grid barrier per PDES epoch).
#pragma once
#include <cstring>
#include <memory>
#include <stdexcept>
#include <map>
#include <string>
#include <vector>

#include "../model/epoch.h"
#include "../power/power_eval.h"
#include "../trace/trace.h"

namespace asim {

struct RunLimits {
  uint64_t max_cycle = 0;   // absolute cycle cap (0 = none)
  uint64_t max_epochs = 0;  // safety cap (0 = none)
};

// In-loop power sampling (power_eval.h): while armed, the engine takes a
// sample at the end of the first epoch reaching `next` (= last sample + freq,
// which also clamps the epoch decision's fast-forward, as a sampled slice's
// max_cycle would) and at every run exit, from its own statistics, with no
// return to the host per sample (reference mcpat_cycle inside the cycle loop,
// power_interface.cc:52-188)
struct PwrArm {
  PwrCoef coef;
  uint64_t freq = 0;
  uint64_t t_prev = 0;           // cycle of the previous sample (arm point)
  double s_prev[PS_COUNT] = {};  // sums at t_prev
  uint32_t n_sm = 0;
};

struct RunResult {
  uint64_t end_cycle = 0;
  uint64_t epochs = 0;
  bool done = false;        // at least one kernel completed (done_mask)
  uint32_t done_mask = 0;   // bit k: the kernel in slot k completed at end_cycle
  bool deadlock = false;
  bool hit_limit = false;
  bool cap = false;  // stopped by -gpgpu_max_insn / -gpgpu_max_cta / -gpgpu_max_completed_cta
};

class Engine {
 public:
  virtual ~Engine() = default;
  virtual const char* name() const = 0;
  virtual void init(const SimCfg& c) = 0;
  // start kernel `k` in free slot `slot` (< kMaxConc; uploads its trace): its
  // CTAs dispatch from kd.ready_cycle on.  `k` must stay alive until the
  // kernel completes.
  virtual void launch(uint32_t slot, ReadyKernel& k, const KernelDesc& kd) = 0;
  // simulate the running kernels until one (or more, same epoch) completes,
  // a limit is hit, or deadlock; completed slots are free again afterwards
  virtual RunResult run(const RunLimits& lim) = 0;
  // bit k: slot k holds a running kernel
  virtual uint32_t running() const = 0;
  // cycle at which the next epoch would start
  virtual uint64_t now() const = 0;
  // L2 pre-fill for MemcpyHtoD (reference perf_memcpy_to_gpu, gpu-sim.cc:2116-2136)
  virtual void memcpy_fill_l2(uint64_t addr, uint64_t bytes) = 0;
  // invalidate the L2s; with `writeback` the dirty sectors are first written
  // to memory (the MALL when there is one), as the release at the end of a
  // kernel does on a multi-XCD GPU
  virtual void flush_l2(bool writeback = false) = 0;
  // DVFS: core cycles from `base_cyc` on last `per_core` fs, cycle base_cyc
  // beginning at femtosecond `base_fs` (called at an epoch boundary, i.e.
  // between run() calls; per_core must not exceed SimCfg::per_core_max)
  virtual void set_core_clock(uint64_t per_core, uint64_t base_cyc, uint64_t base_fs) = 0;
  virtual void stats(std::vector<SMStats>& sm, std::vector<MemStats>& mem) = 0;
  // raw state image (SM states then channel states) for checkpoint/compare
  virtual void snapshot(std::vector<uint8_t>& out) = 0;
  virtual void restore(const std::vector<uint8_t>& in) = 0;
  // advance the clock without simulating (collective stalls, idle time)
  virtual void advance(uint64_t cycles) = 0;
  // complete, engine-independent timing state (SM + channel states, epoch
  // publication block, both mailbox parities, clocks): a checkpoint written
  // by one engine resumes on the other (SURVEY §5.4 timing-state snapshot)
  virtual void save_state(std::vector<uint8_t>& out) = 0;
  virtual void load_state(const std::vector<uint8_t>& in) = 0;
  // debug trace streams: events recorded since the last drain (per unit, in
  // program order); `dropped` counts events lost to full per-unit buffers
  virtual void trace_drain(std::vector<TraceEv>& out, uint64_t* dropped) = 0;
  // kernel-trace residency: peak bytes of trace held by the engine's compute
  // device at once, and how often a window was refilled (GPU engine streaming;
  // host engines report 0)
  virtual void trace_residency(uint64_t* peak_bytes, uint64_t* refills) const {
    *peak_bytes = 0;
    *refills = 0;
  }
  // device kernel launches so far (GPU engine; host engines report 0)
  virtual uint64_t launches() const { return 0; }
  // -icnt_link_contention: packets delayed by busy links, their total delay
  // in interconnect cycles (icnt_links.h), and packets a routing deadlock of
  // the router model left at their uncontended latency (icnt_router.h)
  virtual void link_stats(uint64_t* delayed, uint64_t* wait_cycles, uint64_t* deadlocked = nullptr) {
    *delayed = 0;
    *wait_cycles = 0;
    if (deadlocked) *deadlocked = 0;
  }
  // in-loop power sampling (PwrArm); engines without it return false
  virtual bool power_sampler() const { return false; }
  virtual void power_arm(const PwrArm&) { throw std::runtime_error("engine has no in-loop power sampler"); }
  virtual void power_disarm() {}
  // samples taken since the last drain, in order
  virtual void power_drain(std::vector<PwrSample>& out) { out.clear(); }
};

// host twin of the samplers' step 2 (the sums of every unit's raw counters)
inline void pwr_sums_of(const SMStats* const* sm, size_t nsm, const MemStats* const* mem, size_t nmem, double* S) {
  for (int j = 0; j < PS_COUNT; ++j) S[j] = 0;
  for (size_t i = 0; i < nsm; ++i)
    for (int r = 0; r < PR_COUNT; ++r) {
      const int j = pwr_sum_of(r);
      if (j >= 0) S[j] += (double)pwr_raw_sm(*sm[i], r);
    }
  for (size_t i = 0; i < nmem; ++i)
    for (int r = 0; r < PR_COUNT; ++r) {
      const int j = pwr_sum_of(r);
      if (j >= 0) S[j] += (double)pwr_raw_mem(*mem[i], r);
    }
}

// one sample from the sums at `now` (shared by the engines' samplers)
inline PwrSample pwr_take(PwrArm& a, const double* S, uint64_t now) {
  PwrSample o{};
  double d[PS_COUNT];
  for (int j = 0; j < PS_COUNT; ++j) d[j] = S[j] - a.s_prev[j];
  pwr_activity(d, now > a.t_prev ? (double)(now - a.t_prev) : 1.0, a.n_sm, o);
  pwr_power(a.coef, a.coef.coef, a.n_sm, 1.0, 1.0, 1.0, o);
  o.now = now;
  for (int j = 0; j < PS_COUNT; ++j) a.s_prev[j] = S[j];
  a.t_prev = now;
  return o;
}

// layout of save_state(): header, then SMState[n_sm], ChanState[n_mem],
// EpochPub, and for parity 0/1: req packets, req counts, reply packets,
// reply counts
// capacity of each sub-partition's arrival backlog ring (packets): every SM
// can have at most icnt_out_limit packets in flight, so n_sm of them bound
// what one destination can ever hold back; capped to keep MI355X-sized
// configurations at a few MB per sub-partition
inline uint32_t backlog_cap(const SimCfg& c) {
  uint64_t b = (uint64_t)c.n_sm * c.icnt_out_limit;
  return (uint32_t)(b < 16384 ? b : 16384);
}

struct EngineStateHeader {
  uint64_t magic = 0x41534d5354415445ull;  // "ASMSTATE"
  uint64_t version = 8;  // 4: kernel slots (concurrent kernels); 5: MALL lines; 6: link reservations;
                         // 7: DRAM queue bound (ChanState::q_hi), router deadlock statistics word;
                         // 8: SMState instruction window / packet queues after the hot prefix
  uint64_t n_sm = 0, n_mem = 0, sm_bytes = 0, ch_bytes = 0, pub_bytes = 0;
  uint64_t box_req = 0, cnt_req = 0, box_rep = 0, cnt_rep = 0;  // element counts per parity
  uint64_t ovf = 0;                                              // arrival backlog packets (all sub-partitions)
  uint64_t mall = 0;                                             // MALL lines (all channels), after the backlog
  uint64_t links = 0;  // -icnt_link_contention: link free times, then the two statistics words, after the MALL
  uint64_t cycle = 0, epoch = 0, ready = 0;
};

// helpers for the serialisation
struct StateOut {
  std::vector<uint8_t>& v;
  void put(const void* p, size_t n) {
    const size_t o = v.size();
    v.resize(o + n);
    if (n) memcpy(v.data() + o, p, n);
  }
};
struct StateIn {
  const std::vector<uint8_t>& v;
  size_t off = 0;
  const uint8_t* take(size_t n) {
    if (off + n > v.size()) throw std::runtime_error("engine state: truncated image");
    const uint8_t* p = v.data() + off;
    off += n;
    return p;
  }
  void get(void* dst, size_t n) { memcpy(dst, take(n), n); }
};
void check_state_header(const EngineStateHeader& h, const EngineStateHeader& want);

std::unique_ptr<Engine> make_cpu_engine();
// defined in the HIP engine module; returns nullptr when no GPU is usable
std::unique_ptr<Engine> make_gpu_engine();
bool gpu_engine_available();
// lock-step checker: runs `primary` and `reference` side by side and compares
// their timing-state images every `interval` cycles (check_engine.cc);
// `corrupt_at` (0 = off) perturbs the reference image from that cycle on, to
// test the checker itself (a unit state byte, or with `corrupt_mailbox` the
// first request-mailbox count)
std::unique_ptr<Engine> make_check_engine(std::unique_ptr<Engine> primary, std::unique_ptr<Engine> reference,
                                          uint64_t interval, uint64_t corrupt_at = 0, bool corrupt_mailbox = false);
int gpu_cu_count();  // compute units of the current HIP device (0 if none)
int gpu_cus_per_sim(uint32_t n_sm, uint32_t n_mem);  // CUs one GPU-engine simulation of this shape reserves
std::map<std::string, uint64_t> gpu_pool_stats();  // the GPU engine's caching allocator (empty without HIP)
void gpu_pool_trim();  // give the allocator's cached blocks back to the driver
std::map<std::string, uint64_t> gpu_batch_stats();
std::map<std::string, std::map<std::string, uint64_t>> gpu_engine_modes();  // per engine build: LDS, blocks per CU, registers  // global-state batch launches: batches, launches, blocks per CU
// compiled resources of the persistent engine kernel (empty if no HIP build):
// registers, scratch, static LDS, plus the dynamic LDS the engine requests
struct EngineKernelInfo {
  int num_regs = 0, local_bytes = 0, shared_static = 0, max_threads = 0, binary_version = 0;
  size_t lds_dynamic = 0, sm_state_bytes = 0, chan_state_bytes = 0;
  bool valid = false;
};
EngineKernelInfo gpu_engine_kernel_info();

// MALL lines of one channel (0 without a MALL)
inline uint64_t mall_lines(const SimCfg& c) { return (uint64_t)c.mall_sets * c.mall_assoc; }

// helpers shared by both engines
uint32_t reply_cap(const SimCfg& c);
void check_core_clock(const SimCfg& c, uint64_t per_core);
void host_memcpy_fill(ChanState* chs, uint32_t nch, const SimCfg& c, uint64_t addr, uint64_t bytes);
// mall: the channels' MALL lines [nch][mall_lines(c)] (nullptr without a MALL)
void host_flush_l2(ChanState* chs, uint32_t nch, const SimCfg& c, bool writeback = false, L2Line* mall = nullptr);
void init_sm_state(SMState& s, uint32_t id);
void init_chan_state(ChanState& ch, uint32_t id, const SimCfg& c);

}  // namespace asim
