// MI355X (gfx950) cycle engine, host side (the kernel: engine_kernel.h).
//
// One persistent launch simulates up to `max_epochs` PDES epochs of the whole
// simulated GPU:
//   * block b < n_sm      : one 64-lane wavefront owns SM b; its complete
//                           SMState (~105 KB) lives in LDS for the launch.
//   * block n_sm + c      : one wavefront owns memory channel c (two L2
//                           sub-partitions + the DRAM channel, ~118 KB LDS).
//   * after every epoch   : one grid-wide barrier (agent-scope release /
//                           acquire, XCD-local counters first, then a global
//                           generation word), then every block evaluates the
//                           same epoch decision and all blocks leave together.
// The cycle model itself is the shared single-source code in csrc/model, run
// with the WavePar lane policy, so results are bit-identical to the CPU
// reference engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>

#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <vector>

#include "engine_kernel.h"
#include "trace_window.h"

namespace asim {

#define HIPCHECK(x)                                                                                  \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess)                                                                            \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x);    \
  } while (0)

// builds of engine_kernel, instantiated in the kernel TUs (engine_k_*.hip)
extern template __global__ void engine_kernel<WavePar, false, kModeLds>(GpuArgs);
extern template __global__ void engine_kernel<WavePar, true, kModeLds>(GpuArgs);
extern template __global__ void engine_kernel<WaveParProf, false, kModeLds>(GpuArgs);
extern template __global__ void engine_kernel<WaveParProf, true, kModeLds>(GpuArgs);
extern template __global__ void engine_kernel<WavePar, true, kModeGlobal>(GpuArgs);
extern template __global__ void engine_kernel<WaveParProf, true, kModeGlobal>(GpuArgs);
extern template __global__ void engine_kernel<WavePar, true, kModeSplit>(GpuArgs);
extern template __global__ void engine_kernel<WaveParProf, true, kModeSplit>(GpuArgs);
hipError_t engine_upload_cfg_lds(const SimCfg& c, int slot);
hipError_t engine_upload_cfg_prof(const SimCfg& c, int slot);
hipError_t engine_upload_cfg_global(const SimCfg& c, int slot);
hipError_t engine_upload_cfg_split(const SimCfg& c, int slot);
hipError_t engine_upload_cfg_split2(const SimCfg& c, int slot);

namespace {

// Machine-wide CU reservation between PROCESSES sharing one GPU (job-level
// parallelism: several accel-sim.out / bench ranks per card).  A table of
// (pid, CUs) holders per device in a file under /tmp, guarded by flock; a
// launch waits until the CUs it needs are free, holders that died are pruned.
class DeviceCuTable {
 public:
  struct Ent {
    int32_t pid;
    int32_t cus;
  };
  static constexpr int kMax = 256;
  explicit DeviceCuTable(int dev) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) snprintf(bus, sizeof(bus), "dev%d", dev);
    for (char* q = bus; *q; ++q)
      if (*q == ':' || *q == '.') *q = '_';
    path_ = std::string("/tmp/asim_gpu_cus_") + bus + ".lock";
    fd_ = open(path_.c_str(), O_RDWR | O_CREAT, 0666);
    if (fd_ >= 0) (void)fchmod(fd_, 0666);
  }
  ~DeviceCuTable() {
    if (fd_ >= 0) close(fd_);
  }
  void acquire(int n, int cap) {
    if (fd_ < 0) return;  // no shared table: only the in-process pool applies
    for (int spin = 0;; ++spin) {
      if (flock(fd_, LOCK_EX) != 0) return;
      std::vector<Ent> e = load();
      int used = 0;
      for (const Ent& x : e) used += x.cus;
      if (used + n <= cap || e.empty()) {
        e.push_back(Ent{(int32_t)getpid(), (int32_t)n});
        store(e);
        flock(fd_, LOCK_UN);
        return;
      }
      flock(fd_, LOCK_UN);
      usleep(spin < 100 ? 200 : 2000);
    }
  }
  void release(int n) {
    if (fd_ < 0 || flock(fd_, LOCK_EX) != 0) return;
    std::vector<Ent> e = load();
    for (size_t i = 0; i < e.size(); ++i)
      if (e[i].pid == (int32_t)getpid() && e[i].cus == n) {
        e.erase(e.begin() + (long)i);
        break;
      }
    store(e);
    flock(fd_, LOCK_UN);
  }

 private:
  std::vector<Ent> load() {
    std::vector<Ent> e(kMax);
    const ssize_t r = pread(fd_, e.data(), sizeof(Ent) * kMax, 0);
    e.resize(r > 0 ? (size_t)r / sizeof(Ent) : 0);
    std::vector<Ent> live;
    for (const Ent& x : e)  // drop holders that no longer exist
      if (x.pid > 0 && x.cus > 0 && (kill(x.pid, 0) == 0 || errno == EPERM)) live.push_back(x);
    return live;
  }
  void store(const std::vector<Ent>& e) {
    if (ftruncate(fd_, 0) != 0) return;
    if (!e.empty()) (void)pwrite(fd_, e.data(), sizeof(Ent) * e.size(), 0);
  }
  std::string path_;
  int fd_ = -1;
};

// Engine blocks per CU are accounted in slots, kCuSlots per CU (840 =
// lcm(1..8): any whole number of blocks per CU up to 8 divides it).  An
// LDS-state block takes the share of the CU's LDS it allocates (a whole CU);
// a global-state block takes kCuSlots / (its blocks per CU), the kernel's
// occupancy from its register and LDS use (one block of margin below the
// occupancy API's figure, which can read one block high: MI355X_MICROARCH
// "Occupancy API one block/CU high"), at most 8.
constexpr uint32_t kCuSlots = 840;
constexpr uint32_t kMaxBlocksPerCu = 8;
uint32_t block_slots(size_t lds) {
  const size_t per_cu = lds ? (160 * 1024) / lds : kMaxBlocksPerCu;  // blocks whose LDS fits one CU
  return kCuSlots / (uint32_t)std::max<size_t>(1, std::min<size_t>(per_cu, kMaxBlocksPerCu));
}
// ASIM_GPU_STATE: split (default) | lds | global (engine_kernel.h EngineMode).
// The split build is the default: 5-9 % slower per simulated SM than the
// LDS build but three engine waves per CU instead of one, which measured
// +6.5 % on the node bench, +12 % GPU-engine-only and +11 % on the config
// sweep on one box (profiles/r6/README.md)
int gpu_state_mode() {
  const char* e = getenv("ASIM_GPU_STATE");
  if (!e || !*e) return kModeSplit;
  const std::string v(e);
  return v == "global" ? kModeGlobal : v == "lds" ? kModeLds : kModeSplit;
}
bool gpu_state_global() { return gpu_state_mode() == kModeGlobal; }
// ASIM_GPU_SPLIT_WAVES=2: the split build's two-waves-per-SIMD kernel
// (engine_k_split2.hip); 1 (default): one wave per SIMD, all registers
int split_waves() {
  const char* e = getenv("ASIM_GPU_SPLIT_WAVES");
  return e && atoi(e) == 2 ? 2 : 1;
}
int g_occ_api = 0;  // the occupancy API's blocks per CU of the last mode asked (diagnostics)
// blocks of one mode's kernel per CU (cached per mode; needs a current device)
uint32_t mode_blocks_per_cu(int mode) {
  if (mode == kModeLds) return 1;
  static std::mutex mu;
  static uint32_t cache[3] = {0, 0, 0};
  std::lock_guard<std::mutex> g(mu);
  if (!cache[mode]) {
    int occ = 0;
    const void* f = mode == kModeGlobal ? (const void*)engine_batch_kernel
                    : split_waves() == 2 ? (const void*)engine_split2_kernel
                                         : (const void*)engine_kernel<WavePar, true, kModeSplit>;
    const size_t lds = mode == kModeGlobal ? kLdsBytesGlobal : kLdsBytesSplit;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, f, 64, (int)lds) != hipSuccess) occ = 2;
    g_occ_api = occ;
    occ = occ > 1 ? occ - 1 : 1;
    if (const char* e = getenv("ASIM_GPU_BLOCKS_PER_CU"))  // measured override (co-residency tests)
      if (atoi(e) > 0) occ = atoi(e);
    cache[mode] = (uint32_t)std::min<int>(occ, (int)kMaxBlocksPerCu);
  }
  return cache[mode];
}
uint32_t global_blocks_per_cu() { return mode_blocks_per_cu(kModeGlobal); }
// Blocks of one simulation and, of them, the channels' (GpuArgs::ch_blocks).
// One block per unit while the units fit `cap` blocks; larger configs time-
// slice several units per block.  The split build can pack
// ASIM_GPU_CH_PER_BLOCK channels per block (a GV100 simulation then takes 96
// blocks instead of 112 with 2): off by default -- with the channels in HBM a
// channel pair lengthens the epoch, GPU-engine suite 52.0k -> 42.5k sim KIPS
// at 2 per block (profiles/r6/README.md).
struct BlockPlan {
  uint32_t nblocks, ch_blocks;
};
BlockPlan block_plan(uint32_t n_sm, uint32_t n_mem, int mode, uint32_t cap) {
  BlockPlan p{n_sm + n_mem, 0};
  if (mode == kModeSplit && n_sm > 0 && n_mem > 0) {
    uint32_t pack = 1;
    if (const char* e = getenv("ASIM_GPU_CH_PER_BLOCK"))
      if (atoi(e) > 0) pack = (uint32_t)atoi(e);
    const uint32_t chb = (n_mem + pack - 1) / pack;
    if (pack > 1 && n_sm + chb <= cap) p = BlockPlan{n_sm + chb, chb};
  }
  if (p.nblocks > cap) p = BlockPlan{cap, 0};
  return p;
}
uint32_t engine_block_slots(int mode) { return kCuSlots / mode_blocks_per_cu(mode); }
bool profiling_env() {
  const char* pe = getenv("ASIM_GPU_PROFILE");
  return pe && *pe && *pe != '0';
}
// ASIM_GPU_BATCH=1: global- / split-state simulations of a process share
// batch launches (engine_batch_kernel / engine_batch_split_kernel).  Off by
// default: a batch ends with its slowest simulation and forms only when the
// simulations are in their GPU phase together, and one kernel per simulation
// on the process's hardware queues measured faster (profiles/r6/README.md)
bool gpu_batch_on() {
  const char* e = getenv("ASIM_GPU_BATCH");
  return e && std::string(e) == "1";
}

// Process-wide CU reservation.  Every simulation needs ALL its blocks
// co-resident (grid barrier) and each block takes one CU (LDS-bound), so
// concurrent simulations in one process (job-level parallelism on one GPU)
// must never oversubscribe the CUs: a launch waits until its CUs are free,
// first in this process, then in the machine-wide table of the device.
class CuPool {
 public:
  static CuPool& get() {
    static CuPool p;
    return p;
  }
  void init(int cus) {
    std::lock_guard<std::mutex> g(mu_);
    if (cap_ == 0) {
      cap_ = free_ = cus;
      int dev = 0;
      if (hipGetDevice(&dev) == hipSuccess) table_.reset(new DeviceCuTable(dev));
    }
  }
  void acquire(int n) {
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return free_ >= n; });
      free_ -= n;
    }
    if (table_) table_->acquire(n, cap_);
  }
  void release(int n) {
    if (table_) table_->release(n);
    {
      std::lock_guard<std::mutex> g(mu_);
      free_ += n;
    }
    cv_.notify_all();
  }
  int capacity() {
    std::lock_guard<std::mutex> g(mu_);
    return cap_;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int cap_ = 0, free_ = 0;
  std::unique_ptr<DeviceCuTable> table_;
};

// constant-memory configuration slots (g_cfg) of the engines alive in this
// process: simulations that run at once read their own slot
class CfgSlots {
 public:
  static CfgSlots& get() {
    static CfgSlots s;
    return s;
  }
  int acquire() {
    std::lock_guard<std::mutex> g(mu_);
    for (int i = 0; i < kCfgSlots; ++i)
      if (!(used_ >> i & 1ull)) {
        used_ |= 1ull << i;
        return i;
      }
    throw std::runtime_error("GPU engine: more than 64 simulations alive in one process");
  }
  void release(int i) {
    std::lock_guard<std::mutex> g(mu_);
    used_ &= ~(1ull << i);
  }

 private:
  std::mutex mu_;
  uint64_t used_ = 0;
};


// Process-wide caching allocator for the engine's device buffers, pinned
// control words and streams.  hipFree / hipHostFree / hipStreamDestroy
// synchronise the whole device: with several simulations sharing the GPU
// (the node bench runs GPU-engine applications side by side, and every
// step's simulations are built and torn down again), one simulation's
// teardown waited for the other's running engine_kernel launch -- a queued
// application measured 0.084 s alone and 0.14-0.19 s inside the step.
// Buffers go back to a free list keyed by their exact size and are handed to
// the next simulation of that shape (the bench repeats the same shapes every
// step).  The cache is bounded: a block that would take the cached bytes over
// the cap (ASIM_GPU_POOL_CAP_MB, default 4096 device / 1024 pinned) is freed
// at once, and an allocation that fails first gives every cached block back
// to the driver (one device synchronisation) and retries.
class DevicePool {
 public:
  static DevicePool& get() {
    static DevicePool* p = new DevicePool();  // never destroyed: no frees during static teardown
    return *p;
  }
  struct Stats {
    size_t cached_dev = 0, cached_host = 0, cap_dev = 0, cap_host = 0;
    uint64_t trims = 0, freed_over_cap = 0;
  };
  Stats stats() {
    std::lock_guard<std::mutex> g(mu_);
    Stats t = st_;
    t.cap_dev = cap_dev_;
    t.cap_host = cap_host_;
    return t;
  }
  void* dev(size_t n) {
    if (void* q = take(dev_, n, st_.cached_dev)) return q;
    void* q = nullptr;
    if (hipMalloc(&q, n ? n : 16) != hipSuccess) {
      (void)hipGetLastError();
      trim();
      HIPCHECK(hipMalloc(&q, n ? n : 16));
    }
    std::lock_guard<std::mutex> g(mu_);
    size_[q] = n;
    return q;
  }
  void dev_free(void* q) {
    if (!q) return;
    std::unique_lock<std::mutex> g(mu_);
    auto it = size_.find(q);
    if (it == size_.end()) {  // not ours (never happens): give it back
      g.unlock();
      (void)hipFree(q);
      return;
    }
    if (st_.cached_dev + it->second > cap_dev_) {  // over the cap: back to the driver
      size_.erase(it);
      ++st_.freed_over_cap;
      g.unlock();
      (void)hipFree(q);
      return;
    }
    st_.cached_dev += it->second;
    dev_[it->second].push_back(q);
  }
  void* host(size_t n) {
    if (void* q = take(host_, n, st_.cached_host)) return q;
    void* q = nullptr;
    if (hipHostMalloc(&q, n ? n : 16) != hipSuccess) {
      (void)hipGetLastError();
      trim();
      HIPCHECK(hipHostMalloc(&q, n ? n : 16));
    }
    std::lock_guard<std::mutex> g(mu_);
    hsize_[q] = n;
    return q;
  }
  void host_free(void* q) {
    if (!q) return;
    std::unique_lock<std::mutex> g(mu_);
    auto it = hsize_.find(q);
    if (it == hsize_.end()) {
      g.unlock();
      (void)hipHostFree(q);
      return;
    }
    if (st_.cached_host + it->second > cap_host_) {
      hsize_.erase(it);
      ++st_.freed_over_cap;
      g.unlock();
      (void)hipHostFree(q);
      return;
    }
    st_.cached_host += it->second;
    host_[it->second].push_back(q);
  }
  // every cached block back to the driver (the frees synchronise the device)
  void trim() {
    std::map<size_t, std::vector<void*>> d, h;
    {
      std::lock_guard<std::mutex> g(mu_);
      d.swap(dev_);
      h.swap(host_);
      for (auto& kv : d)
        for (void* q : kv.second) size_.erase(q);
      for (auto& kv : h)
        for (void* q : kv.second) hsize_.erase(q);
      st_.cached_dev = st_.cached_host = 0;
      ++st_.trims;
    }
    (void)hipDeviceSynchronize();
    for (auto& kv : d)
      for (void* q : kv.second) (void)hipFree(q);
    for (auto& kv : h)
      for (void* q : kv.second) (void)hipHostFree(q);
  }
  hipStream_t stream() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!streams_.empty()) {
        hipStream_t s = streams_.back();
        streams_.pop_back();
        return s;
      }
    }
    hipStream_t s = nullptr;
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  void stream_free(hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> g(mu_);
    streams_.push_back(s);
  }

 private:
  DevicePool() {
    size_t mb = 4096;
    if (const char* e = getenv("ASIM_GPU_POOL_CAP_MB")) mb = (size_t)strtoull(e, nullptr, 10);
    cap_dev_ = mb << 20;
    cap_host_ = std::min<size_t>(cap_dev_, (size_t)1024 << 20);
  }
  void* take(std::map<size_t, std::vector<void*>>& m, size_t n, size_t& cached) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = m.find(n);
    if (it == m.end() || it->second.empty()) return nullptr;
    void* q = it->second.back();
    it->second.pop_back();
    cached -= n;
    return q;
  }
  std::mutex mu_;
  std::map<size_t, std::vector<void*>> dev_, host_;
  std::map<void*, size_t> size_, hsize_;
  std::vector<hipStream_t> streams_;
  size_t cap_dev_ = 0, cap_host_ = 0;
  Stats st_;
};
template <class T>
void pool_alloc(T** p, size_t n) {
  *p = static_cast<T*>(DevicePool::get().dev(n));
}

// Batch launches of the global-state engine (job-level parallelism on ONE
// GPU, the reference's run_simulations.py / procman.py fan-out of
// independent simulations, util/job_launching/run_simulations.py:375-397).
// A process can only run a few kernels at once (GPU_MAX_HW_QUEUES hardware
// queues), while a global-state simulation needs one wave per unit and an
// MI355X holds several per CU.  So the simulations of a process submit their
// launches here; a submitting thread becomes a leader and packs the pending
// launches that fit the free CU slots into ONE engine_batch_kernel, and each
// simulation's blocks synchronise only with each other (own GpuCtl).  Up to
// kMaxBatches batches run at once, each on its own stream.  (More than one
// is not safe with the global-state kernel: it spills ~1 KB per lane to
// scratch, and batches on several hardware queues then failed to keep all
// their waves resident -- a grid barrier timed out with at most 512 blocks
// in flight over up to three queues where one queue held 672:
// profiles/r6/README.md.)  A leader waits
// until every simulation inside run() has submitted, or kBatchWaitUs after
// the oldest pending launch (a simulation between two of its launches is
// usually back within that).  Launches are capped at kBatchEpochs epochs so
// a short one does not wait long for a long one of its batch.
class BatchLauncher {
 public:
  static constexpr uint32_t kBatchEpochs = 1024;
  static constexpr int kBatchWaitUs = 2000;
  static constexpr int kMaxBatches = 1;  // concurrent batches
  static BatchLauncher& get() {
    static BatchLauncher* b = new BatchLauncher();  // never destroyed
    return *b;
  }
  struct Sub {
    GpuArgs a;
    int mode = kModeGlobal;  // kModeGlobal or kModeSplit: a batch holds one build
    uint32_t nb = 0, slots = 0;
    GpuCtl* h_ctl = nullptr;
    bool done = false;
    hipError_t err = hipSuccess;
  };
  // simulations currently inside GpuEngine::run (the leader waits for them)
  void enter() {
    std::lock_guard<std::mutex> g(mu_);
    ++in_run_;
  }
  void leave() {
    std::lock_guard<std::mutex> g(mu_);
    --in_run_;
    cv_.notify_all();
  }
  void run(Sub& me) {
    std::unique_lock<std::mutex> g(mu_);
    pending_.push_back(&me);
    if (pending_.size() == 1) first_ = std::chrono::steady_clock::now();
    cv_.notify_all();
    while (!me.done) {
      const bool queued = std::find(pending_.begin(), pending_.end(), &me) != pending_.end();
      if (queued && running_ < kMaxBatches) {
        // every simulation inside run() that is not in a running batch has submitted
        const bool all_in = (int)pending_.size() >= in_run_ - in_flight_;
        const bool waited = std::chrono::steady_clock::now() - first_ >= std::chrono::microseconds(kBatchWaitUs);
        if (all_in || waited) {
          lead(g);
          continue;
        }
        cv_.wait_for(g, std::chrono::microseconds(25));
        continue;
      }
      cv_.wait(g);
    }
  }
  uint64_t batches() const { return batches_; }
  uint64_t jobs() const { return jobs_; }

 private:
  struct Slot {  // one batch's stream and job tables
    hipStream_t stream = nullptr;
    GpuArgs *d_jobs = nullptr, *h_jobs = nullptr;
    uint16_t *d_bj = nullptr, *h_bj = nullptr;
    size_t jobs_cap = 0, blocks_cap = 0;
    bool busy = false;
  };
  void lead(std::unique_lock<std::mutex>& g) {
    Slot* sl = nullptr;
    for (Slot& x : slots_)
      if (!x.busy) {
        sl = &x;
        break;
      }
    sl->busy = true;
    ++running_;
    // FIFO: the pending launches that fit the GPU's slots (at least one)
    const uint32_t cap = (uint32_t)CuPool::get().capacity();
    std::vector<Sub*> take;
    uint32_t slots = 0, blocks = 0;
    const int mode = pending_.front()->mode;
    for (auto it = pending_.begin(); it != pending_.end();) {
      Sub* x = *it;
      if (x->mode != mode) {
        ++it;
        continue;
      }
      if (!take.empty() && (slots + x->nb * x->slots > cap || blocks + x->nb > 65535u)) break;
      take.push_back(x);
      slots += x->nb * x->slots;
      blocks += x->nb;
      it = pending_.erase(it);
    }
    in_flight_ += (int)take.size();
    if (!pending_.empty()) first_ = std::chrono::steady_clock::now();
    g.unlock();
    hipError_t err = launch(*sl, take, blocks, slots, mode);
    g.lock();
    for (Sub* x : take) {
      x->err = err;
      x->done = true;
    }
    in_flight_ -= (int)take.size();
    ++batches_;
    jobs_ += take.size();
    sl->busy = false;
    --running_;
    // the launches that waited behind this batch now wait (up to
    // kBatchWaitUs) for its simulations to come back, so the next batch
    // takes them together instead of alternating with them
    if (!pending_.empty()) first_ = std::chrono::steady_clock::now();
    cv_.notify_all();
  }
  hipError_t launch(Slot& sl, std::vector<Sub*>& take, uint32_t blocks, uint32_t slots, int mode) {
    if (!sl.stream) {
      if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) return hipErrorOutOfMemory;
    }
    const size_t njobs = take.size();
    if (njobs > sl.jobs_cap || blocks > sl.blocks_cap) {
      const size_t nj = std::max<size_t>(njobs, 2 * sl.jobs_cap), nbk = std::max<size_t>(blocks, 2 * sl.blocks_cap);
      (void)hipFree(sl.d_jobs);
      (void)hipFree(sl.d_bj);
      (void)hipHostFree(sl.h_jobs);
      (void)hipHostFree(sl.h_bj);
      sl.d_jobs = sl.h_jobs = nullptr;
      sl.d_bj = sl.h_bj = nullptr;
      hipError_t e = hipMalloc(&sl.d_jobs, sizeof(GpuArgs) * nj);
      if (e == hipSuccess) e = hipMalloc(&sl.d_bj, sizeof(uint16_t) * nbk);
      if (e == hipSuccess) e = hipHostMalloc(&sl.h_jobs, sizeof(GpuArgs) * nj);
      if (e == hipSuccess) e = hipHostMalloc(&sl.h_bj, sizeof(uint16_t) * nbk);
      if (e != hipSuccess) {
        sl.jobs_cap = sl.blocks_cap = 0;
        return e;
      }
      sl.jobs_cap = nj;
      sl.blocks_cap = nbk;
    }
    uint32_t b0 = 0;
    for (size_t j = 0; j < njobs; ++j) {
      GpuArgs a = take[j]->a;
      a.block0 = b0;
      sl.h_jobs[j] = a;
      for (uint32_t i = 0; i < take[j]->nb; ++i) sl.h_bj[b0 + i] = (uint16_t)j;
      b0 += take[j]->nb;
    }
    hipError_t e = hipMemcpyAsync(sl.d_jobs, sl.h_jobs, sizeof(GpuArgs) * njobs, hipMemcpyHostToDevice, sl.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(sl.d_bj, sl.h_bj, sizeof(uint16_t) * blocks, hipMemcpyHostToDevice, sl.stream);
    for (size_t j = 0; j < njobs && e == hipSuccess; ++j) e = hipMemsetAsync(take[j]->a.ctl, 0, sizeof(GpuCtl), sl.stream);
    if (e != hipSuccess) return e;
    CuPool::get().acquire((int)slots);
    if (mode == kModeSplit)
      hipLaunchKernelGGL(engine_batch_split_kernel, dim3(blocks), dim3(64), kLdsBytesSplit, sl.stream,
                         (const GpuArgs*)sl.d_jobs, (const uint16_t*)sl.d_bj);
    else
      hipLaunchKernelGGL(engine_batch_kernel, dim3(blocks), dim3(64), kLdsBytesGlobal, sl.stream,
                         (const GpuArgs*)sl.d_jobs, (const uint16_t*)sl.d_bj);
    e = hipGetLastError();
    for (size_t j = 0; j < njobs; ++j) {
      const hipError_t ce =
          hipMemcpyAsync(take[j]->h_ctl, take[j]->a.ctl, sizeof(GpuCtl), hipMemcpyDeviceToHost, sl.stream);
      if (e == hipSuccess) e = ce;
    }
    const hipError_t se = hipStreamSynchronize(sl.stream);
    CuPool::get().release((int)slots);
    return e != hipSuccess ? e : se;
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Sub*> pending_;
  std::chrono::steady_clock::time_point first_;
  int running_ = 0;    // batches in flight
  int in_flight_ = 0;  // launches in those batches
  int in_run_ = 0;
  Slot slots_[kMaxBatches];
  uint64_t batches_ = 0, jobs_ = 0;
};

class GpuEngine : public Engine {
 public:
  ~GpuEngine() override {
    try {
      dump_profile();
    } catch (...) {
    }
    DevicePool::get().dev_free(d_prof_);
    DevicePool::get().dev_free(d_ework_);
    release();
    if (cfg_slot_ >= 0) CfgSlots::get().release(cfg_slot_);
  }
  const char* name() const override { return "gpu"; }

  void init(const SimCfg& c) override {
    c_ = c;
    int dev = 0;
    HIPCHECK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, dev));
    n_cu_ = prop.multiProcessorCount;
    CuPool::get().init(n_cu_ * kCuSlots);
    // one block per unit while the units fit the CUs; larger configs (or a
    // smaller ASIM_GPU_BLOCKS cap) time-slice several units per block
    mode_ = gpu_state_mode();
    uint32_t cap = (uint32_t)n_cu_ * mode_blocks_per_cu(mode_);
    if (const char* eb = getenv("ASIM_GPU_BLOCKS"))
      if (atoi(eb) > 0) cap = std::min<uint32_t>(cap, (uint32_t)atoi(eb));
    const BlockPlan bp = block_plan(c.n_sm, c.n_mem, mode_, cap);
    nblocks_ = bp.nblocks;
    ch_blocks_ = bp.ch_blocks;
    global_ = mode_ == kModeGlobal;
    lds_ = global_ ? kLdsBytesGlobal : mode_ == kModeSplit ? kLdsBytesSplit : kLdsBytes;
    sliced_ = nblocks_ < c.n_sm + c.n_mem;
    for (const void* f : {(const void*)engine_kernel<WavePar, false, kModeLds>, (const void*)engine_kernel<WaveParProf, false, kModeLds>,
                          (const void*)engine_kernel<WavePar, true, kModeLds>, (const void*)engine_kernel<WaveParProf, true, kModeLds>})
      HIPCHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes));
    // every block of a simulation must be co-resident: a block takes the CU
    // slots (kCuSlots per CU) its LDS needs, one at least
    slots_ = engine_block_slots(mode_);
    batch_ = (global_ || mode_ == kModeSplit) && !profiling_env() && gpu_batch_on();
    if (cfg_slot_ < 0) cfg_slot_ = CfgSlots::get().acquire();
    const char* pe = getenv("ASIM_GPU_PROFILE");
    profiling_ = pe && *pe && *pe != '0';
    if (profiling_) {
      pool_alloc(&d_prof_, sizeof(uint64_t) * nblocks_ * kProfSlots);
      HIPCHECK(hipMemset(d_prof_, 0, sizeof(uint64_t) * nblocks_ * kProfSlots));
      pool_alloc(&d_ework_, sizeof(uint32_t) * nblocks_);
    }
    stream_ = DevicePool::get().stream();
    if (!done_ev_) HIPCHECK(hipEventCreateWithFlags(&done_ev_, hipEventBlockingSync | hipEventDisableTiming));
    if (c_.trace_mask) {
      // debug trace buffers in HBM; the device copy of the config points at them
      const size_t units = (size_t)c.n_sm + c.n_mem;
      pool_alloc(&d_trace_ev_, units * c_.trace_cap * sizeof(TraceEv));
      pool_alloc(&d_trace_cnt_, units * sizeof(uint32_t));
      HIPCHECK(hipMemset(d_trace_cnt_, 0, units * sizeof(uint32_t)));
      c_.trace_ev = d_trace_ev_;
      c_.trace_cnt = d_trace_cnt_;
    }
    pool_alloc(&d_cfg_, sizeof(SimCfg));
    upload_cfg();
    std::vector<SMState> hs(c.n_sm);
    for (uint32_t i = 0; i < c.n_sm; ++i) init_sm_state(hs[i], i);
    std::vector<ChanState> hc(c.n_mem);
    for (uint32_t i = 0; i < c.n_mem; ++i) init_chan_state(hc[i], i, c);
    pool_alloc(&d_sms_, sizeof(SMState) * c.n_sm);
    pool_alloc(&d_chs_, sizeof(ChanState) * c.n_mem);
    HIPCHECK(hipMemcpy(d_sms_, hs.data(), sizeof(SMState) * c.n_sm, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_chs_, hc.data(), sizeof(ChanState) * c.n_mem, hipMemcpyHostToDevice));
    pool_alloc(&d_pub_, sizeof(EpochPub));
    HIPCHECK(hipMemset(d_pub_, 0, sizeof(EpochPub)));
    cap_req_ = c.icnt_latency;
    cap_rep_ = reply_cap(c);
    for (int p = 0; p < 2; ++p) {
      // mailboxes start zeroed (like the CPU engine's) so state images and
      // checkpoints never carry uninitialised device memory
      pool_alloc(&d_box_req_[p], sizeof(Pkt) * c.n_subpart * c.n_sm * cap_req_);
      HIPCHECK(hipMemset(d_box_req_[p], 0, sizeof(Pkt) * c.n_subpart * c.n_sm * cap_req_));
      pool_alloc(&d_cnt_req_[p], sizeof(uint32_t) * c.n_subpart * c.n_sm);
      HIPCHECK(hipMemset(d_cnt_req_[p], 0, sizeof(uint32_t) * c.n_subpart * c.n_sm));
      pool_alloc(&d_box_rep_[p], sizeof(Pkt) * c.n_sm * c.n_subpart * cap_rep_);
      HIPCHECK(hipMemset(d_box_rep_[p], 0, sizeof(Pkt) * c.n_sm * c.n_subpart * cap_rep_));
      pool_alloc(&d_cnt_rep_[p], sizeof(uint32_t) * c.n_sm * c.n_subpart);
      HIPCHECK(hipMemset(d_cnt_rep_[p], 0, sizeof(uint32_t) * c.n_sm * c.n_subpart));
    }
    ovf_cap_ = backlog_cap(c);
    pool_alloc(&d_ovf_, sizeof(Pkt) * c.n_subpart * (size_t)ovf_cap_);
    HIPCHECK(hipMemset(d_ovf_, 0, sizeof(Pkt) * c.n_subpart * (size_t)ovf_cap_));
    n_mall_ = (size_t)c.n_mem * mall_lines(c);
    if (n_mall_) {
      pool_alloc(&d_mall_, sizeof(L2Line) * n_mall_);
      HIPCHECK(hipMemset(d_mall_, 0, sizeof(L2Line) * n_mall_));
    }
    if (c.link_contention && (icnt_link_count(c) > kMaxIcntLinks || !icnt_contention_fits(c, cap_req_, cap_rep_) ||
                              icnt_scratch_words(c, cap_req_, cap_rep_) > kMaxIcntScratchWords))
      throw std::runtime_error("-icnt_link_contention: topology or mailboxes too large for the link pass");
    n_links_ = icnt_contention_on(c) ? (size_t)icnt_state_words(c, cap_req_, cap_rep_) : 0;
    if (n_links_) {
      pool_alloc(&d_links_, sizeof(uint64_t) * (n_links_ + kIcntStatWords));
      HIPCHECK(hipMemset(d_links_, 0, sizeof(uint64_t) * (n_links_ + kIcntStatWords)));
      pool_alloc(&d_link_refs_, sizeof(uint32_t) * (size_t)icnt_scratch_words(c, cap_req_, cap_rep_));
    }
    pool_alloc(&d_ctl_, sizeof(GpuCtl));
    h_ctl_ = static_cast<GpuCtl*>(DevicePool::get().host(sizeof(GpuCtl)));
    pool_alloc(&d_kt_, sizeof(KernelTab));
    kt_ = KernelTab{};
    kt_.mix = c.concurrent_kernel_sm;
    epoch_ = 0;
    cycle_ = 0;
  }

  void launch(uint32_t slot, ReadyKernel& k, const KernelDesc& kd) override {
    if (slot >= (uint32_t)kMaxConc || (kt_.active >> slot & 1u)) throw std::runtime_error("launch: kernel slot busy");
    if (!k.streamed() && k.insts.size() > kIdxMask) throw std::runtime_error("kernel trace exceeds 2^29 warp instructions");
    KernelDesc& d = kt_.k[slot];
    d = kd;
    // whole kernel uploaded, or (-gpu_trace_window / host-streamed trace) a
    // window of CTAs that follows the dispatch cursor (trace_window.h)
    tw_.launch(slot, k, d, c_);
    kt_.active |= 1u << slot;
  }
  uint32_t running() const override { return kt_.active; }

  RunResult run(const RunLimits& lim) override {
    RunResult res;
    if (!kt_.active) {
      res.end_cycle = cycle_;
      return res;
    }
    // batch mode: this simulation counts as one the batch leader waits for
    struct InRun {
      bool on;
      explicit InRun(bool b) : on(b) {
        if (on) BatchLauncher::get().enter();
      }
      ~InRun() {
        if (on) BatchLauncher::get().leave();
      }
    } in_run(batch_);
    for (;;) {
      tw_.ensure(kt_, c_, [&](DispatchView& v) { read_dispatch(v); });
      HIPCHECK(hipMemcpy(d_kt_, &kt_, sizeof(KernelTab), hipMemcpyHostToDevice));
      GpuArgs a{};
      a.cfg_slot = (uint32_t)cfg_slot_;
      a.cfg_g = d_cfg_;
      a.kt = d_kt_;
      a.sms = d_sms_;
      a.chs = d_chs_;
      a.pub = d_pub_;
      for (int p = 0; p < 2; ++p) {
        a.box_req[p] = d_box_req_[p];
        a.cnt_req[p] = d_cnt_req_[p];
        a.box_rep[p] = d_box_rep_[p];
        a.cnt_rep[p] = d_cnt_rep_[p];
      }
      a.cap_req = cap_req_;
      a.cap_rep = cap_rep_;
      a.ovf = d_ovf_;
      a.ovf_cap = ovf_cap_;
      a.mall = d_mall_;
      a.link_free = d_links_;
      a.link_refs = d_link_refs_;
      a.epoch0 = epoch_;
      a.cycle0 = cycle_;
      a.max_cycle = lim.max_cycle;
      a.max_epochs = epochs_per_launch_;
      a.nblocks = nblocks_;
      a.ch_blocks = ch_blocks_;
      a.ctl = d_ctl_;
      HIPCHECK(hipMemsetAsync(d_ctl_, 0, sizeof(GpuCtl), stream_));
      a.prof = d_prof_;
      a.ework = d_ework_;
      a.pw = pw_on_ ? d_pw_ : nullptr;
      if (batch_) {
        // the launch joins the process's next batch (BatchLauncher)
        a.max_epochs = std::min<uint32_t>(a.max_epochs, BatchLauncher::kBatchEpochs);
        BatchLauncher::Sub sub;
        sub.a = a;
        sub.mode = mode_;
        sub.nb = nblocks_;
        sub.slots = slots_;
        sub.h_ctl = h_ctl_;
        BatchLauncher::get().run(sub);
        ++launches_;
        HIPCHECK(sub.err);
      } else {
      CuPool::get().acquire((int)(nblocks_ * slots_));
      hipError_t le;
      if (mode_ == kModeSplit && profiling_)
        hipLaunchKernelGGL((engine_kernel<WaveParProf, true, kModeSplit>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (mode_ == kModeSplit && split_waves() == 2)
        hipLaunchKernelGGL(engine_split2_kernel, dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (mode_ == kModeSplit)
        hipLaunchKernelGGL((engine_kernel<WavePar, true, kModeSplit>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (global_ && profiling_)
        hipLaunchKernelGGL((engine_kernel<WaveParProf, true, kModeGlobal>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (global_)
        hipLaunchKernelGGL((engine_kernel<WavePar, true, kModeGlobal>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (profiling_ && sliced_)
        hipLaunchKernelGGL((engine_kernel<WaveParProf, true, kModeLds>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (profiling_)
        hipLaunchKernelGGL((engine_kernel<WaveParProf, false, kModeLds>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else if (sliced_)
        hipLaunchKernelGGL((engine_kernel<WavePar, true, kModeLds>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      else
        hipLaunchKernelGGL((engine_kernel<WavePar, false, kModeLds>), dim3(nblocks_), dim3(64), lds_, stream_, a);
      le = hipGetLastError();
      ++launches_;
      hipError_t ce = hipMemcpyAsync(h_ctl_, d_ctl_, sizeof(GpuCtl), hipMemcpyDeviceToHost, stream_);
      // wait on a blocking-sync event: the host thread sleeps instead of
      // spinning, so simulations waiting on the GPU leave the host cores to
      // the CPU-engine simulations of the node schedule
      hipError_t se = hipEventRecord(done_ev_, stream_);
      if (se == hipSuccess) se = hipEventSynchronize(done_ev_);
      CuPool::get().release((int)(nblocks_ * slots_));
      HIPCHECK(le);
      HIPCHECK(ce);
      HIPCHECK(se);
      }
      if (h_ctl_->error) throw std::runtime_error("GPU engine: grid barrier timed out (blocks not co-resident?)");
      epoch_ = h_ctl_->end_epoch;
      cycle_ = h_ctl_->end_cycle;
      if (pw_on_) pwr_collect();
      res.epochs += h_ctl_->epochs_run;
      if (h_ctl_->done) {
        res.done = true;
        res.done_mask = h_ctl_->done;
        kt_.active &= ~h_ctl_->done;
        for (uint32_t s = 0; s < (uint32_t)kMaxConc; ++s)
          if (h_ctl_->done >> s & 1u) tw_.done(s);
        break;
      }
      if (h_ctl_->deadlock) { res.deadlock = true; break; }
      if (h_ctl_->cap) { res.hit_limit = true; res.cap = true; break; }
      if ((lim.max_cycle && cycle_ >= lim.max_cycle) || (lim.max_epochs && res.epochs >= lim.max_epochs)) {
        res.hit_limit = true;
        break;
      }
      if (h_ctl_->epochs_run == 0) throw std::runtime_error("GPU engine made no progress");
    }
    res.end_cycle = cycle_;
    return res;
  }

  uint64_t now() const override { return cycle_; }

  void memcpy_fill_l2(uint64_t addr, uint64_t bytes) override {
    std::vector<ChanState> hc(c_.n_mem);
    HIPCHECK(hipMemcpy(hc.data(), d_chs_, sizeof(ChanState) * c_.n_mem, hipMemcpyDeviceToHost));
    host_memcpy_fill(hc.data(), c_.n_mem, c_, addr, bytes);
    HIPCHECK(hipMemcpy(d_chs_, hc.data(), sizeof(ChanState) * c_.n_mem, hipMemcpyHostToDevice));
  }
  void set_core_clock(uint64_t per_core, uint64_t base_cyc, uint64_t base_fs) override {
    check_core_clock(c_, per_core);
    c_.per_core = per_core;
    c_.clk_base_cyc = base_cyc;
    c_.clk_base_fs = base_fs;
    cfg_set_divs(c_);
    upload_cfg();
  }
  void flush_l2(bool writeback) override {
    std::vector<ChanState> hc(c_.n_mem);
    HIPCHECK(hipMemcpy(hc.data(), d_chs_, sizeof(ChanState) * c_.n_mem, hipMemcpyDeviceToHost));
    std::vector<L2Line> hm(writeback ? n_mall_ : 0);
    if (!hm.empty()) HIPCHECK(hipMemcpy(hm.data(), d_mall_, sizeof(L2Line) * n_mall_, hipMemcpyDeviceToHost));
    host_flush_l2(hc.data(), c_.n_mem, c_, writeback, hm.empty() ? nullptr : hm.data());
    HIPCHECK(hipMemcpy(d_chs_, hc.data(), sizeof(ChanState) * c_.n_mem, hipMemcpyHostToDevice));
    if (!hm.empty()) HIPCHECK(hipMemcpy(d_mall_, hm.data(), sizeof(L2Line) * n_mall_, hipMemcpyHostToDevice));
  }

  void stats(std::vector<SMStats>& sm, std::vector<MemStats>& mem) override {
    sm.resize(c_.n_sm);
    HIPCHECK(hipMemcpy2D(sm.data(), sizeof(SMStats), reinterpret_cast<char*>(d_sms_) + offsetof(SMState, st),
                         sizeof(SMState), sizeof(SMStats), c_.n_sm, hipMemcpyDeviceToHost));
    mem.clear();
    for (uint32_t j = 0; j < c_.n_sub_per_mem; ++j) {
      std::vector<MemStats> part(c_.n_mem);
      size_t off = offsetof(ChanState, sp) + j * sizeof(SubPart) + offsetof(SubPart, st);
      HIPCHECK(hipMemcpy2D(part.data(), sizeof(MemStats), reinterpret_cast<char*>(d_chs_) + off, sizeof(ChanState),
                           sizeof(MemStats), c_.n_mem, hipMemcpyDeviceToHost));
      if (j == 0) mem.resize((size_t)c_.n_mem * c_.n_sub_per_mem);
      for (uint32_t i = 0; i < c_.n_mem; ++i) mem[(size_t)i * c_.n_sub_per_mem + j] = part[i];
    }
  }

  void snapshot(std::vector<uint8_t>& out) override {
    const size_t units = sizeof(SMState) * c_.n_sm + sizeof(ChanState) * c_.n_mem;
    out.resize(units + sizeof(L2Line) * n_mall_ + 8 * n_links_);
    HIPCHECK(hipMemcpy(out.data(), d_sms_, sizeof(SMState) * c_.n_sm, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(out.data() + sizeof(SMState) * c_.n_sm, d_chs_, sizeof(ChanState) * c_.n_mem,
                       hipMemcpyDeviceToHost));
    if (n_mall_) HIPCHECK(hipMemcpy(out.data() + units, d_mall_, sizeof(L2Line) * n_mall_, hipMemcpyDeviceToHost));
    if (n_links_)
      HIPCHECK(hipMemcpy(out.data() + units + sizeof(L2Line) * n_mall_, d_links_, 8 * n_links_, hipMemcpyDeviceToHost));
  }
  void restore(const std::vector<uint8_t>& in) override {
    const size_t units = sizeof(SMState) * c_.n_sm + sizeof(ChanState) * c_.n_mem;
    if (in.size() != units + sizeof(L2Line) * n_mall_ + 8 * n_links_) throw std::runtime_error("snapshot size mismatch");
    HIPCHECK(hipMemcpy(d_sms_, in.data(), sizeof(SMState) * c_.n_sm, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_chs_, in.data() + sizeof(SMState) * c_.n_sm, sizeof(ChanState) * c_.n_mem,
                       hipMemcpyHostToDevice));
    if (n_mall_) HIPCHECK(hipMemcpy(d_mall_, in.data() + units, sizeof(L2Line) * n_mall_, hipMemcpyHostToDevice));
    if (n_links_)
      HIPCHECK(hipMemcpy(d_links_, in.data() + units + sizeof(L2Line) * n_mall_, 8 * n_links_, hipMemcpyHostToDevice));
  }
  void link_stats(uint64_t* delayed, uint64_t* wait_cycles, uint64_t* deadlocked) override {
    uint64_t st[kIcntStatWords] = {};
    if (n_links_) HIPCHECK(hipMemcpy(st, d_links_ + n_links_, sizeof(st), hipMemcpyDeviceToHost));
    *delayed = st[0];
    *wait_cycles = st[1];
    if (deadlocked) *deadlocked = st[2];
  }
  void advance(uint64_t cycles) override {
    uint64_t E = c_.icnt_latency;
    cycle_ += (cycles + E - 1) / E * E;
  }
  void set_epochs_per_launch(uint32_t n) { epochs_per_launch_ = n ? n : 4096; }

  void trace_drain(std::vector<TraceEv>& out, uint64_t* dropped) override {
    out.clear();
    if (!c_.trace_mask) return;
    const size_t units = (size_t)c_.n_sm + c_.n_mem;
    std::vector<uint32_t> cnt(units);
    HIPCHECK(hipMemcpy(cnt.data(), d_trace_cnt_, units * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (size_t u = 0; u < units; ++u) {
      const uint32_t k = std::min(cnt[u], c_.trace_cap);
      if (dropped) *dropped += cnt[u] - k;
      if (!k) continue;
      const size_t o = out.size();
      out.resize(o + k);
      HIPCHECK(hipMemcpy(out.data() + o, d_trace_ev_ + u * c_.trace_cap, k * sizeof(TraceEv), hipMemcpyDeviceToHost));
    }
    HIPCHECK(hipMemset(d_trace_cnt_, 0, units * sizeof(uint32_t)));
  }

  // same image layout as the CPU engine (engine.h EngineStateHeader), so a
  // state saved here resumes on either engine
  EngineStateHeader header() const {
    EngineStateHeader h;
    h.n_sm = c_.n_sm;
    h.n_mem = c_.n_mem;
    h.sm_bytes = sizeof(SMState);
    h.ch_bytes = sizeof(ChanState);
    h.pub_bytes = sizeof(EpochPub);
    h.box_req = (uint64_t)c_.n_subpart * c_.n_sm * cap_req_;
    h.cnt_req = (uint64_t)c_.n_subpart * c_.n_sm;
    h.box_rep = (uint64_t)c_.n_sm * c_.n_subpart * cap_rep_;
    h.cnt_rep = (uint64_t)c_.n_sm * c_.n_subpart;
    h.ovf = (uint64_t)c_.n_subpart * ovf_cap_;
    h.mall = n_mall_;
    h.links = n_links_ ? n_links_ + kIcntStatWords : 0;
    h.cycle = cycle_;
    h.epoch = epoch_;
    h.ready = kt_.active;
    return h;
  }
  void save_state(std::vector<uint8_t>& out) override {
    const EngineStateHeader h = header();
    out.assign(sizeof(h), 0);
    memcpy(out.data(), &h, sizeof(h));
    auto dl = [&](const void* d, size_t n) {
      const size_t o = out.size();
      out.resize(o + n);
      if (n) HIPCHECK(hipMemcpy(out.data() + o, d, n, hipMemcpyDeviceToHost));
    };
    dl(d_sms_, sizeof(SMState) * c_.n_sm);
    dl(d_chs_, sizeof(ChanState) * c_.n_mem);
    dl(d_pub_, sizeof(EpochPub));
    for (int p = 0; p < 2; ++p) {
      dl(d_box_req_[p], h.box_req * sizeof(Pkt));
      dl(d_cnt_req_[p], h.cnt_req * sizeof(uint32_t));
      dl(d_box_rep_[p], h.box_rep * sizeof(Pkt));
      dl(d_cnt_rep_[p], h.cnt_rep * sizeof(uint32_t));
    }
    dl(d_ovf_, h.ovf * sizeof(Pkt));
    dl(d_mall_, h.mall * sizeof(L2Line));
    dl(d_links_, h.links * sizeof(uint64_t));  // free times + the two statistics words (CPU engine layout)
  }
  void load_state(const std::vector<uint8_t>& in) override {
    StateIn r{in};
    EngineStateHeader h;
    r.get(&h, sizeof(h));
    const EngineStateHeader w = header();
    check_state_header(h, w);
    auto ul = [&](void* d, size_t n) {
      if (n) HIPCHECK(hipMemcpy(d, r.take(n), n, hipMemcpyHostToDevice));
    };
    ul(d_sms_, sizeof(SMState) * c_.n_sm);
    ul(d_chs_, sizeof(ChanState) * c_.n_mem);
    ul(d_pub_, sizeof(EpochPub));
    for (int p = 0; p < 2; ++p) {
      ul(d_box_req_[p], w.box_req * sizeof(Pkt));
      ul(d_cnt_req_[p], w.cnt_req * sizeof(uint32_t));
      ul(d_box_rep_[p], w.box_rep * sizeof(Pkt));
      ul(d_cnt_rep_[p], w.cnt_rep * sizeof(uint32_t));
    }
    ul(d_ovf_, w.ovf * sizeof(Pkt));
    ul(d_mall_, w.mall * sizeof(L2Line));
    ul(d_links_, w.links * sizeof(uint64_t));
    cycle_ = h.cycle;
    epoch_ = h.epoch;
    if (h.ready) throw std::runtime_error("engine state: image taken with kernels running");
  }

 private:
  // samples of the last launch from the device ring; the ring restarts
  void pwr_collect() {
    uint32_t n = 0;
    HIPCHECK(hipMemcpy(&n, reinterpret_cast<char*>(d_pw_) + offsetof(PwrDev, n), sizeof(n), hipMemcpyDeviceToHost));
    if (n > pw_cap_) throw std::runtime_error("GPU engine: power sample ring overflow");
    if (n) {
      const size_t o = pw_out_.size();
      pw_out_.resize(o + n);
      HIPCHECK(hipMemcpy(pw_out_.data() + o, d_pw_ring_, sizeof(PwrSample) * n, hipMemcpyDeviceToHost));
      const uint32_t z = 0;
      HIPCHECK(hipMemcpy(reinterpret_cast<char*>(d_pw_) + offsetof(PwrDev, n), &z, sizeof(z), hipMemcpyHostToDevice));
    }
  }

  // the dispatch state a trace window follows: replicated cursors (SM 0) and
  // every SM's resident CTAs, read back from the device
  void read_dispatch(DispatchView& v) {
    const size_t off_d = offsetof(SMState, k_uid);
    const size_t len_d = offsetof(SMState, next_ctax) + sizeof(SMState::next_ctax) - off_d;
    std::vector<char> disp(len_d);
    HIPCHECK(hipMemcpy(disp.data(), reinterpret_cast<char*>(d_sms_) + off_d, len_d, hipMemcpyDeviceToHost));
    memcpy(v.k_uid, disp.data() + (offsetof(SMState, k_uid) - off_d), sizeof(v.k_uid));
    memcpy(v.next_cta, disp.data() + (offsetof(SMState, next_cta) - off_d), sizeof(v.next_cta));
    memcpy(v.next_ctax, disp.data() + (offsetof(SMState, next_ctax) - off_d), sizeof(v.next_ctax));
    const size_t off_c = offsetof(SMState, cta_id);
    const size_t len_c = offsetof(SMState, cta_wbase) - off_c;
    std::vector<char> ctas((size_t)c_.n_sm * len_c);
    HIPCHECK(hipMemcpy2D(ctas.data(), len_c, reinterpret_cast<char*>(d_sms_) + off_c, sizeof(SMState), len_c, c_.n_sm,
                         hipMemcpyDeviceToHost));
    v.sms.resize(c_.n_sm);
    for (uint32_t m = 0; m < c_.n_sm; ++m) {
      const char* e = ctas.data() + (size_t)m * len_c;
      memcpy(v.sms[m].cta_id, e, sizeof(v.sms[m].cta_id));
      memcpy(v.sms[m].cta_valid, e + (offsetof(SMState, cta_valid) - off_c), sizeof(v.sms[m].cta_valid));
      memcpy(v.sms[m].cta_ks, e + (offsetof(SMState, cta_ks) - off_c), sizeof(v.sms[m].cta_ks));
    }
  }

 public:
  void trace_residency(uint64_t* peak_bytes, uint64_t* refills) const override {
    *peak_bytes = tw_.resident_peak;
    *refills = tw_.refills;
  }

  // in-kernel power sampling (engine.h PwrArm): engine_kernel writes each
  // sample to a device ring, drained after every launch
  uint64_t launches() const override { return launches_; }
  bool power_sampler() const override { return true; }
  void power_arm(const PwrArm& arm) override {
    const uint32_t nunits = c_.n_sm + c_.n_mem;
    const uint32_t cap = epochs_per_launch_ + 2;  // at most one sample per epoch of a launch
    if (!d_pw_) pool_alloc(&d_pw_, sizeof(PwrDev));
    if (!d_pw_rows_) pool_alloc(&d_pw_rows_, sizeof(double) * kPwrRawPad * nunits);
    if (pw_cap_ < cap) {
      DevicePool::get().dev_free(d_pw_ring_);
      pool_alloc(&d_pw_ring_, sizeof(PwrSample) * cap);
      pw_cap_ = cap;
    }
    PwrDev h{};
    h.coef = arm.coef;
    h.freq = arm.freq;
    h.t_prev = arm.t_prev;
    h.next = arm.t_prev + arm.freq;
    h.n_sm = arm.n_sm;
    h.n = 0;
    h.cap = pw_cap_;
    for (int j = 0; j < PS_COUNT; ++j) h.s_prev[j] = arm.s_prev[j];
    h.rows = d_pw_rows_;
    h.ring = d_pw_ring_;
    HIPCHECK(hipMemcpy(d_pw_, &h, sizeof(PwrDev), hipMemcpyHostToDevice));
    pw_on_ = true;
    pw_out_.clear();
  }
  void power_disarm() override { pw_on_ = false; }
  void power_drain(std::vector<PwrSample>& out) override {
    out.swap(pw_out_);
    pw_out_.clear();
  }

 private:
  // the configuration as the kernels read it: the engine's constant-memory
  // slot and the global copy (stream-ordered before the next launch)
  void upload_cfg() {
    HIPCHECK(hipMemcpy(d_cfg_, &c_, sizeof(SimCfg), hipMemcpyHostToDevice));
    HIPCHECK(engine_upload_cfg_lds(c_, cfg_slot_));
    HIPCHECK(engine_upload_cfg_prof(c_, cfg_slot_));
    HIPCHECK(engine_upload_cfg_global(c_, cfg_slot_));
    HIPCHECK(engine_upload_cfg_split(c_, cfg_slot_));
    HIPCHECK(engine_upload_cfg_split2(c_, cfg_slot_));
  }
  void release() {
    auto fr = [](void* p) {
      DevicePool::get().dev_free(p);
    };
    fr(d_cfg_);
    fr(d_sms_);
    fr(d_chs_);
    fr(d_pub_);
    for (int p = 0; p < 2; ++p) {
      fr(d_box_req_[p]);
      fr(d_cnt_req_[p]);
      fr(d_box_rep_[p]);
      fr(d_cnt_rep_[p]);
    }
    fr(d_ctl_);
    fr(d_ovf_);
    fr(d_mall_);
    fr(d_links_);
    fr(d_link_refs_);
    n_links_ = 0;
    fr(d_trace_ev_);
    fr(d_trace_cnt_);
    tw_.release();
    fr(d_pw_);
    fr(d_pw_rows_);
    fr(d_pw_ring_);
    fr(d_kt_);
    DevicePool::get().host_free(h_ctl_);
    DevicePool::get().stream_free(stream_);
    if (done_ev_) (void)hipEventDestroy(done_ev_);
    done_ev_ = nullptr;
  }

  SimCfg c_{};
  int cfg_slot_ = -1;
  int n_cu_ = 0;
  uint32_t nblocks_ = 0;
  uint32_t ch_blocks_ = 0;  // blocks of the packed channels (block_plan)
  size_t lds_ = 0;
  hipStream_t stream_ = nullptr;
  hipEvent_t done_ev_ = nullptr;  // blocking-sync event the launch waits on
  SimCfg* d_cfg_ = nullptr;
  SMState* d_sms_ = nullptr;
  ChanState* d_chs_ = nullptr;
  EpochPub* d_pub_ = nullptr;
  Pkt* d_ovf_ = nullptr;  // arrival backlog rings [n_subpart][ovf_cap_]
  L2Line* d_mall_ = nullptr;  // MALL lines [n_mem][mall_sets * mall_assoc]
  size_t n_mall_ = 0;
  uint64_t* d_links_ = nullptr;     // -icnt_link_contention: link free times + 2 statistics words
  uint32_t* d_link_refs_ = nullptr;
  size_t n_links_ = 0;
  uint32_t ovf_cap_ = 0;
  Pkt* d_box_req_[2] = {nullptr, nullptr};
  uint32_t* d_cnt_req_[2] = {nullptr, nullptr};
  Pkt* d_box_rep_[2] = {nullptr, nullptr};
  uint32_t* d_cnt_rep_[2] = {nullptr, nullptr};
  GpuCtl* d_ctl_ = nullptr;
  GpuCtl* h_ctl_ = nullptr;
  TraceEv* d_trace_ev_ = nullptr;
  uint32_t* d_trace_cnt_ = nullptr;
  // device rings / whole copies of the running kernels' traces
  struct DevMem {
    static constexpr bool kHost = false;
    void* alloc(size_t n) {
      void* p = nullptr;
      pool_alloc(&p, n);
      return p;
    }
    void free(void* p) {
      DevicePool::get().dev_free(p);
    }
    void write(void* d, const void* h, size_t n) { HIPCHECK(hipMemcpy(d, h, n, hipMemcpyHostToDevice)); }
  };
  TraceWindows<DevMem> tw_;
  uint64_t launches_ = 0;
  bool pw_on_ = false;
  PwrDev* d_pw_ = nullptr;
  double* d_pw_rows_ = nullptr;
  PwrSample* d_pw_ring_ = nullptr;
  uint32_t pw_cap_ = 0;
  std::vector<PwrSample> pw_out_;
  KernelTab kt_{};
  KernelTab* d_kt_ = nullptr;
  uint32_t cap_req_ = 0, cap_rep_ = 0;
  uint64_t epoch_ = 0, cycle_ = 0;
  uint32_t epochs_per_launch_ = 4096;
  bool profiling_ = false;
  bool sliced_ = false;  // more units than blocks: the time-slicing kernel
  int mode_ = kModeLds;  // ASIM_GPU_STATE (EngineMode)
  bool global_ = false;  // ASIM_GPU_STATE=global: unit states stay in HBM (no LDS state)
  bool batch_ = false;   // launches shared with the process's other global-state simulations (BatchLauncher)
  uint32_t slots_ = kCuSlots;  // CU slots one block of this engine takes
  uint64_t* d_prof_ = nullptr;
  uint32_t* d_ework_ = nullptr;

 public:
  // per-stage shader-clock totals: [0] = mean over SM blocks, [1] = mean over channel blocks
  void dump_profile() {
    if (!profiling_) return;
    std::vector<uint64_t> h((size_t)nblocks_ * kProfSlots);
    HIPCHECK(hipMemcpy(h.data(), d_prof_, h.size() * 8, hipMemcpyDeviceToHost));
    static const char* names[kProfSlots] = {
        "sm.receive", "sm.writeback", "sm.hit_complete", "sm.ldst", "sm.dispatch", "sm.read_operands",
        "sm.alloc_oc", "sm.issue", "sm.fetch", "sm.retire", "sm.inject", "sm.occupancy", "sm.gather",
        "sm.cta_dispatch", "sm.refill", "sm.cycle_loop", "sm.publish", "#sm_cycles", "#quiet_checks", "#epochs_busy", "mem.gather", "mem.dram",
        "mem.l2", "mem.icnt", "mem.window_other", "mem.publish", "barrier", "decide", "post", "sm.issue_sched", "#slowest", "launch_rest",
        "#max_work/epoch", "#epochs(b0)", "#last_arriver_wait", "#last_arrivals", "ldst.l1_probe", "ldst.mshr_find",
        "ldst.pend_reg", "ldst.send", "recv.xbar", "recv.l1_fill", "issue.one", "issue.pick", "quiet_check", "skip",
        "ldst.hit_push", "fill.pend_wake", "iss.pick", "iss.classify", "iss.step1", "iss.step2", "iss.step3",
        "iss.spare53", "iss.spare54", "iss.spare55"};
    double sm[kProfSlots] = {}, mc[kProfSlots] = {}, smt = 0, mct = 0;
    for (uint32_t b = 0; b < nblocks_; ++b)
      for (int k = 0; k < kProfSlots; ++k) {
        double v = (double)h[(size_t)b * kProfSlots + k];
        const bool counter = (k >= 17 && k <= 19) || k == 30 || (k >= 32 && k <= 35);
        if (b < c_.n_sm) { sm[k] += v / c_.n_sm; smt += counter ? 0 : v / c_.n_sm; }
        else { const double nmb = nblocks_ > c_.n_sm ? (double)(nblocks_ - c_.n_sm) : 1.0; mc[k] += v / nmb; mct += counter ? 0 : v / nmb; }
      }
    // per simulated SM cycle: the SM-cycle stages (slots 0..11) over all SM blocks
    {
      double cyc_clk = 0, n_cyc = 0, n_q = 0, n_ep = 0, q_clk = 0;
      for (uint32_t b = 0; b < c_.n_sm; ++b) {
        for (int k = 0; k <= 11; ++k) cyc_clk += (double)h[(size_t)b * kProfSlots + k];
        for (int k = 36; k <= 43; ++k) cyc_clk += (double)h[(size_t)b * kProfSlots + k];
        cyc_clk += (double)h[(size_t)b * kProfSlots + 29] + (double)h[(size_t)b * kProfSlots + 46] +
                   (double)h[(size_t)b * kProfSlots + 47];
        for (int k = 48; k <= 52; ++k) cyc_clk += (double)h[(size_t)b * kProfSlots + k];
        q_clk += (double)h[(size_t)b * kProfSlots + 44] + (double)h[(size_t)b * kProfSlots + 45];
        n_cyc += (double)h[(size_t)b * kProfSlots + 17];
        n_q += (double)h[(size_t)b * kProfSlots + 18];
        n_ep += (double)h[(size_t)b * kProfSlots + 19];
      }
      fprintf(stderr, "[asim gpu profile] SM cycles simulated %.0f (%.0f clocks each), quiet checks %.0f "
                      "(cycle_loop %.0f clocks each), busy SM-epochs %.0f\n",
              n_cyc, n_cyc ? cyc_clk / n_cyc : 0, n_q, n_q ? q_clk / n_q : 0, n_ep);
    }
    {
      double mx = 0, ne = 0, lw = 0, nl = 0;
      for (uint32_t b = 0; b < nblocks_; ++b) {
        mx += (double)h[(size_t)b * kProfSlots + 32];
        ne += (double)h[(size_t)b * kProfSlots + 33];
        lw += (double)h[(size_t)b * kProfSlots + 34];
        nl += (double)h[(size_t)b * kProfSlots + 35];
      }
      fprintf(stderr, "[asim gpu profile] epochs %.0f: slowest block's work %.0f clocks/epoch; last arriver's "
                      "barrier wait %.0f clocks/epoch (pure barrier latency)\n",
              ne, ne ? mx / ne : 0, nl ? lw / nl : 0);
    }
    {
      std::vector<std::pair<uint64_t, uint32_t>> sl;
      for (uint32_t b = 0; b < nblocks_; ++b) sl.push_back({h[(size_t)b * kProfSlots + 30], b});
      std::sort(sl.rbegin(), sl.rend());
      fprintf(stderr, "[asim gpu profile] slowest block per epoch (epochs, block, its SM cycles / quiet checks):");
      for (size_t i = 0; i < sl.size() && i < 8 && sl[i].first; ++i)
        fprintf(stderr, " %llu x b%u (%s, %llu/%llu)", (unsigned long long)sl[i].first, sl[i].second,
                sl[i].second < c_.n_sm ? "SM" : "MEM", (unsigned long long)h[(size_t)sl[i].second * kProfSlots + 17],
                (unsigned long long)h[(size_t)sl[i].second * kProfSlots + 18]);
      fprintf(stderr, "\n");
    }
    // the critical block: most time outside the barrier wait
    uint32_t crit = 0;
    double crit_work = -1;
    for (uint32_t b = 0; b < nblocks_; ++b) {
      double w = 0;
      for (int k = 0; k < kProfSlots; ++k)
        if (k != 26 && k != 30 && !(k >= 17 && k <= 19) && !(k >= 32 && k <= 35)) w += (double)h[(size_t)b * kProfSlots + k];
      if (w > crit_work) { crit_work = w; crit = b; }
    }
    fprintf(stderr, "[asim gpu profile] shader-clock cycles per block (mean), share of block time; "
                    "CRIT = block %u (%s), the one with the least barrier wait\n", crit, crit < c_.n_sm ? "SM" : "MEM");
    double ct = 0;
    for (int k = 0; k < kProfSlots; ++k)
      if (k != 30 && !(k >= 17 && k <= 19) && !(k >= 32 && k <= 35)) ct += (double)h[(size_t)crit * kProfSlots + k];
    for (int k = 0; k < kProfSlots; ++k) {
      const double cv = (double)h[(size_t)crit * kProfSlots + k];
      if (sm[k] + mc[k] > 0)
        fprintf(stderr, "  %-18s SM %14.0f (%5.1f%%)   MEM %14.0f (%5.1f%%)   CRIT %14.0f (%5.1f%%)\n", names[k], sm[k],
                100 * sm[k] / smt, mc[k], 100 * mc[k] / mct, cv, 100 * cv / ct);
    }
  }

};

}  // namespace

bool gpu_engine_available() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return false;
  return n > 0;
}

std::unique_ptr<Engine> make_gpu_engine() {
  if (!gpu_engine_available()) return nullptr;
  return std::unique_ptr<Engine>(new GpuEngine());
}

}  // namespace asim

namespace asim {
// the engine's caching allocator: cached bytes, caps, trims (tests)
std::map<std::string, uint64_t> gpu_pool_stats() {
  const DevicePool::Stats t = DevicePool::get().stats();
  return {{"cached_dev", t.cached_dev}, {"cached_host", t.cached_host}, {"cap_dev", t.cap_dev},
          {"cap_host", t.cap_host}, {"trims", t.trims}, {"freed_over_cap", t.freed_over_cap}};
}
void gpu_pool_trim() { DevicePool::get().trim(); }
// per engine build: LDS bytes per block, blocks per CU (occupancy API less
// the margin), registers and scratch of its kernel
std::map<std::string, std::map<std::string, uint64_t>> gpu_engine_modes() {
  std::map<std::string, std::map<std::string, uint64_t>> out;
  const struct {
    const char* name;
    int mode;
    const void* f;
    size_t lds;
  } ms[] = {{"lds", kModeLds, (const void*)engine_kernel<WavePar, false, kModeLds>, kLdsBytes},
            {"global", kModeGlobal, (const void*)engine_batch_kernel, kLdsBytesGlobal},
            {"split", kModeSplit, (const void*)engine_kernel<WavePar, true, kModeSplit>, kLdsBytesSplit},
            {"split2", kModeSplit, (const void*)engine_split2_kernel, kLdsBytesSplit}};
  for (const auto& m : ms) {
    auto& o = out[m.name];
    o["lds_bytes"] = m.lds;
    o["blocks_per_cu"] = mode_blocks_per_cu(m.mode);
    int occ = 0;
    if (m.mode == kModeLds) (void)hipFuncSetAttribute(m.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, m.f, 64, (int)m.lds) == hipSuccess) o["occupancy_api"] = occ;
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, m.f) == hipSuccess) {
      o["num_regs"] = (uint64_t)fa.numRegs;
      o["scratch_bytes_per_lane"] = (uint64_t)fa.localSizeBytes;
    }
  }
  out["split"]["sm_hot_bytes"] = kSmHotBytes;
  out["lds"]["sm_state_bytes"] = sizeof(SMState);
  return out;
}
std::map<std::string, uint64_t> gpu_batch_stats() {
  std::map<std::string, uint64_t> m{{"batches", BatchLauncher::get().batches()},
                                     {"launches", BatchLauncher::get().jobs()},
                                     {"blocks_per_cu", global_blocks_per_cu()},
                                     {"occupancy_api", (uint64_t)g_occ_api}};
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, (const void*)engine_batch_kernel) == hipSuccess) {
    m["num_regs"] = (uint64_t)fa.numRegs;
    m["scratch_bytes_per_lane"] = (uint64_t)fa.localSizeBytes;
  }
  return m;
}
// CUs one simulation of this shape reserves on the GPU engine (the
// concurrency of job-level parallelism on one GPU, multi_gpu.py)
int gpu_cus_per_sim(uint32_t n_sm, uint32_t n_mem) {
  const int m = gpu_state_mode();
  const int cus = gpu_cu_count();
  uint32_t cap = cus > 0 ? (uint32_t)cus * mode_blocks_per_cu(m) : n_sm + n_mem;
  if (const char* eb = getenv("ASIM_GPU_BLOCKS"))
    if (atoi(eb) > 0) cap = std::min<uint32_t>(cap, (uint32_t)atoi(eb));
  const uint32_t nb = block_plan(n_sm, n_mem, m, cap).nblocks;
  const uint32_t slots = nb * engine_block_slots(m);
  return (int)((slots + kCuSlots - 1) / kCuSlots);
}
int gpu_cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return p.multiProcessorCount;
}
}  // namespace asim

namespace asim {
EngineKernelInfo gpu_engine_kernel_info() {
  EngineKernelInfo k;
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, (const void*)engine_kernel<WavePar, false, kModeLds>) != hipSuccess) return k;
  k.num_regs = fa.numRegs;
  k.local_bytes = (int)fa.localSizeBytes;
  k.shared_static = (int)fa.sharedSizeBytes;
  k.max_threads = fa.maxThreadsPerBlock;
  k.binary_version = fa.binaryVersion;
  k.lds_dynamic = kLdsBytes;
  k.sm_state_bytes = sizeof(SMState);
  k.chan_state_bytes = sizeof(ChanState);
  k.valid = true;
  return k;
}
}  // namespace asim
