// Persistent host thread team for the CPU engine's epochs (-sim_cpu_threads).
//
// A PDES epoch is 8 simulated cycles (icnt_latency): its units' work is tens
// to hundreds of microseconds, so fork/join per epoch (an OpenMP parallel
// region, ~5-10 us with dynamic scheduling) ate the gain -- 8 OpenMP threads
// measured slower than one on bfs.  This team is the host twin of the GPU
// engine's persistent kernel: the threads stay inside the epoch loop for a
// whole engine run, meet at one spin barrier per epoch, and every thread
// evaluates the (pure) epoch decision itself from the published state, as
// every workgroup of engine_kernel does after its grid barrier.
//
// Between runs the workers park: a short spin, then a condition variable, so
// a team left idle (the driver between kernels, other simulations sharing the
// host) burns no cores.  Spinning waits yield after a bound, so an
// oversubscribed host degrades instead of livelocking.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace asim {

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

class SpinBarrier {
 public:
  explicit SpinBarrier(uint32_t n = 1) : n_(n) {}
  void reset(uint32_t n) {
    n_ = n;
    count_.store(0, std::memory_order_relaxed);
  }
  void wait() {
    const uint32_t g = gen_.load(std::memory_order_acquire);
    if (count_.fetch_add(1, std::memory_order_acq_rel) == n_ - 1) {
      count_.store(0, std::memory_order_relaxed);
      gen_.store(g + 1, std::memory_order_release);
      return;
    }
    uint32_t spins = 0;
    while (gen_.load(std::memory_order_acquire) == g) {
      if (++spins < 4096) cpu_relax();
      else std::this_thread::yield();
    }
  }

 private:
  alignas(64) std::atomic<uint32_t> count_{0};
  alignas(64) std::atomic<uint32_t> gen_{0};
  uint32_t n_;
};

class ThreadTeam {
 public:
  ~ThreadTeam() { stop(); }
  uint32_t size() const { return (uint32_t)workers_.size() + 1; }

  // run job(tid) on tid = 0 (the caller) .. n-1 and return when all finished
  void run(uint32_t n, const std::function<void(uint32_t)>& job) {
    if (n <= 1) {
      job(0);
      return;
    }
    if (size() != n) {
      stop();
      start(n);
    }
    job_ = &job;
    left_.store(n - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    job(0);
    uint32_t spins = 0;
    while (left_.load(std::memory_order_acquire) != 0) {
      if (++spins < 4096) cpu_relax();
      else std::this_thread::yield();
    }
    job_ = nullptr;
  }

 private:
  void start(uint32_t n) {
    quit_ = false;
    // the generation the workers start from is taken here, before run()
    // bumps it: a worker scheduled late must not miss its first job
    const uint32_t g0 = gen_.load(std::memory_order_acquire);
    for (uint32_t t = 1; t < n; ++t) workers_.emplace_back([this, t, g0] { loop(t, g0); });
  }
  void stop() {
    if (workers_.empty()) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
    workers_.clear();
  }
  void loop(uint32_t tid, uint32_t seen) {
    for (;;) {
      // park: spin briefly (back-to-back runs), then sleep
      uint32_t spins = 0;
      while (gen_.load(std::memory_order_acquire) == seen && ++spins < 20000) cpu_relax();
      if (gen_.load(std::memory_order_acquire) == seen) {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_.load(std::memory_order_acquire) != seen; });
      }
      seen = gen_.load(std::memory_order_acquire);
      if (quit_) return;
      (*job_)(tid);
      left_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<uint32_t> gen_{0};
  std::atomic<uint32_t> left_{0};
  const std::function<void(uint32_t)>* job_ = nullptr;
  bool quit_ = false;
};

}  // namespace asim
