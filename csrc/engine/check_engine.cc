// Lock-step engine checker (`-sim_engine check`).
//
// the reference has no race detection; its determinism rests on
// a single host thread.  Here the cycle model runs as hundreds of concurrent
// wavefronts (csrc/engine/gpu_engine.hip) or OpenMP threads
// (cpu_engine.cc), made race-free by the two-phase epoch design
// (csrc/model/epoch.h).  This engine drives the GPU engine and the CPU engine
// side by side over the same kernel, stops both every `-sim_check_interval`
// cycles and compares their complete timing-state images (save_state: every
// SM and channel state, the epoch publication block, both mailbox parities,
// the arrival backlog rings, the clocks) byte for byte.  The first divergence
// aborts the run with the cycle and the unit whose state differs, which
// `-sim_check_interval 1` narrows to one epoch.  Compared: the header, every
// SMState and ChanState, the epoch publication block, every mailbox count of
// both parities, the live packets [0, count) of every mailbox cell, and the
// occupied part of every sub-partition's backlog ring.  Only mailbox slots
// past a cell's count (dead storage) are skipped.
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "engine.h"

namespace asim {
namespace {

class CheckEngine final : public Engine {
 public:
  CheckEngine(std::unique_ptr<Engine> a, std::unique_ptr<Engine> b, uint64_t every, uint64_t corrupt_at,
              bool corrupt_mailbox)
      : a_(std::move(a)), b_(std::move(b)), every_(every ? every : 1), corrupt_at_(corrupt_at),
        corrupt_mailbox_(corrupt_mailbox) {}
  const char* name() const override { return "check"; }
  void init(const SimCfg& c) override {
    n_sm_ = c.n_sm;
    n_mem_ = c.n_mem;
    n_sub_per_mem_ = c.n_sub_per_mem;
    a_->init(c);
    b_->init(c);
  }
  void launch(uint32_t slot, ReadyKernel& k, const KernelDesc& kd) override {
    // both engines would drive one host stream with different windows
    if (k.streamed()) throw std::runtime_error("check engine: host-streamed traces (-trace_host_budget_mb) not supported");
    a_->launch(slot, k, kd);
    b_->launch(slot, k, kd);
  }
  uint32_t running() const override { return a_->running(); }
  void trace_residency(uint64_t* peak_bytes, uint64_t* refills) const override {
    b_->trace_residency(peak_bytes, refills);
  }
  RunResult run(const RunLimits& lim) override {
    RunResult total;
    for (;;) {
      uint64_t cap = a_->now() + every_;
      const bool final_cap = lim.max_cycle && lim.max_cycle <= cap;
      if (final_cap) cap = lim.max_cycle;
      RunLimits l{cap, lim.max_epochs};
      const RunResult ra = a_->run(l);
      const RunResult rb = b_->run(l);
      total.epochs += ra.epochs;
      compare(ra, rb);
      if (ra.done || ra.deadlock || !ra.hit_limit || final_cap || ra.cap) {
        total.end_cycle = ra.end_cycle;
        total.done = ra.done;
        total.done_mask = ra.done_mask;
        total.deadlock = ra.deadlock;
        total.hit_limit = ra.hit_limit;
        total.cap = ra.cap;
        return total;
      }
    }
  }
  uint64_t now() const override { return a_->now(); }
  void memcpy_fill_l2(uint64_t addr, uint64_t bytes) override {
    a_->memcpy_fill_l2(addr, bytes);
    b_->memcpy_fill_l2(addr, bytes);
  }
  void set_core_clock(uint64_t per_core, uint64_t base_cyc, uint64_t base_fs) override {
    a_->set_core_clock(per_core, base_cyc, base_fs);
    b_->set_core_clock(per_core, base_cyc, base_fs);
  }
  void flush_l2(bool writeback) override {
    a_->flush_l2(writeback);
    b_->flush_l2(writeback);
  }
  void stats(std::vector<SMStats>& sm, std::vector<MemStats>& mem) override { a_->stats(sm, mem); }
  void snapshot(std::vector<uint8_t>& out) override { a_->snapshot(out); }
  void restore(const std::vector<uint8_t>& in) override {
    a_->restore(in);
    b_->restore(in);
  }
  void advance(uint64_t cycles) override {
    a_->advance(cycles);
    b_->advance(cycles);
  }
  void save_state(std::vector<uint8_t>& out) override { a_->save_state(out); }
  void load_state(const std::vector<uint8_t>& in) override {
    a_->load_state(in);
    b_->load_state(in);
  }
  void trace_drain(std::vector<TraceEv>& out, uint64_t* dropped) override {
    a_->trace_drain(out, dropped);
    std::vector<TraceEv> discard;
    uint64_t d = 0;
    b_->trace_drain(discard, &d);
  }

 private:
  void compare(const RunResult& ra, const RunResult& rb) {
    ++checks_;
    const uint64_t cyc = a_->now();
    if (ra.end_cycle != rb.end_cycle || ra.done_mask != rb.done_mask || ra.deadlock != rb.deadlock ||
        ra.hit_limit != rb.hit_limit || cyc != b_->now())
      fail(cyc, "run results differ: " + std::string(a_->name()) + " end " + std::to_string(ra.end_cycle) +
                    " done " + std::to_string(ra.done) + ", " + b_->name() + " end " + std::to_string(rb.end_cycle) +
                    " done " + std::to_string(rb.done));
    a_->save_state(ia_);
    b_->save_state(ib_);
    // fault injection for the checker's own test: perturb the reference image
    if (corrupt_at_ && cyc >= corrupt_at_ && ib_.size() > sizeof(EngineStateHeader) + 64) {
      if (corrupt_mailbox_) {
        // first request-mailbox count of parity 0 (right behind the epoch block)
        const size_t o = sizeof(EngineStateHeader) + (size_t)n_sm_ * sizeof(SMState) + (size_t)n_mem_ * sizeof(ChanState) +
                         sizeof(EpochPub);
        EngineStateHeader h;
        memcpy(&h, ib_.data(), sizeof(h));
        const size_t cnt0 = o + h.box_req * sizeof(Pkt);
        if (cnt0 < ib_.size()) ib_[cnt0] ^= 0x01;
      } else {
        ib_[sizeof(EngineStateHeader) + 64] ^= 0x5a;
      }
    }
    const size_t head = sizeof(EngineStateHeader), sm_end = head + (size_t)n_sm_ * sizeof(SMState),
                 ch_end = sm_end + (size_t)n_mem_ * sizeof(ChanState), pub_end = ch_end + sizeof(EpochPub);
    if (ia_.size() != ib_.size() || ia_.size() < pub_end)
      fail(cyc, "state images differ in size (" + std::to_string(ia_.size()) + " vs " + std::to_string(ib_.size()) + ")");
    for (size_t i = 0; i < pub_end; ++i)
      if (ia_[i] != ib_[i]) {
        std::string where = i < head     ? "header"
                            : i < sm_end ? "SM " + std::to_string((i - head) / sizeof(SMState)) + " +" +
                                               std::to_string((i - head) % sizeof(SMState))
                            : i < ch_end ? "channel " + std::to_string((i - sm_end) / sizeof(ChanState)) + " +" +
                                               std::to_string((i - sm_end) % sizeof(ChanState))
                                         : "epoch block +" + std::to_string(i - ch_end);
        diverge(cyc, where, ia_[i], ib_[i]);
      }
    compare_mailboxes(cyc, pub_end);
  }

  // Mailboxes and backlog rings (layout: engine.h save_state).  Counts are
  // compared whole; packets only inside each cell's count; backlog entries
  // only inside each ring's [head, head + n) (head/n are part of ChanState,
  // already equal).
  void compare_mailboxes(uint64_t cyc, size_t off) {
    EngineStateHeader h;
    memcpy(&h, ia_.data(), sizeof(h));
    const uint64_t cap_req = h.cnt_req ? h.box_req / h.cnt_req : 0, cap_rep = h.cnt_rep ? h.box_rep / h.cnt_rep : 0;
    const size_t need = off + 2 * ((h.box_req + h.box_rep) * sizeof(Pkt) + (h.cnt_req + h.cnt_rep) * 4) +
                        h.ovf * sizeof(Pkt) + h.mall * sizeof(L2Line);
    if (ia_.size() < need) fail(cyc, "state image truncated before the mailboxes");
    auto cells = [&](const char* what, int parity, uint64_t nbox, uint64_t ncnt, uint64_t cap) {
      const size_t box = off, cnt = off + nbox * sizeof(Pkt);
      for (uint64_t c = 0; c < ncnt; ++c) {
        uint32_t na, nb;
        memcpy(&na, ia_.data() + cnt + c * 4, 4);
        memcpy(&nb, ib_.data() + cnt + c * 4, 4);
        if (na != nb)
          fail(cyc, std::string(what) + " mailbox count diverges (parity " + std::to_string(parity) + ", cell " +
                        std::to_string(c) + ": " + a_->name() + " " + std::to_string(na) + ", " + b_->name() + " " +
                        std::to_string(nb) + ")");
        const uint64_t live = na < cap ? na : cap;
        const size_t p0 = box + c * cap * sizeof(Pkt);
        for (size_t i = p0; i < p0 + live * sizeof(Pkt); ++i)
          if (ia_[i] != ib_[i])
            diverge(cyc, std::string(what) + " mailbox parity " + std::to_string(parity) + " cell " + std::to_string(c) +
                             " packet " + std::to_string((i - p0) / sizeof(Pkt)) + " +" +
                             std::to_string((i - p0) % sizeof(Pkt)),
                    ia_[i], ib_[i]);
      }
      off = cnt + ncnt * 4;
    };
    for (int p = 0; p < 2; ++p) {
      cells("request", p, h.box_req, h.cnt_req, cap_req);
      cells("reply", p, h.box_rep, h.cnt_rep, cap_rep);
    }
    // backlog rings: [n_subpart][ovf_cap]
    const size_t sm_end = sizeof(EngineStateHeader) + (size_t)n_sm_ * sizeof(SMState);
    const uint64_t nsub = (uint64_t)n_mem_ * n_sub_per_mem_;
    const uint64_t ovf_cap = nsub ? h.ovf / nsub : 0;
    for (uint64_t g = 0; g < nsub && ovf_cap; ++g) {
      const uint64_t ch = g / n_sub_per_mem_, j = g % n_sub_per_mem_;
      const size_t sp = sm_end + ch * sizeof(ChanState) + offsetof(ChanState, sp) + j * sizeof(SubPart);
      uint32_t head_, n_;
      memcpy(&head_, ia_.data() + sp + offsetof(SubPart, ovf_head), 4);
      memcpy(&n_, ia_.data() + sp + offsetof(SubPart, ovf_n), 4);
      for (uint32_t k = 0; k < n_ && k < ovf_cap; ++k) {
        const size_t p0 = off + (g * ovf_cap + (head_ + k) % ovf_cap) * sizeof(Pkt);
        for (size_t i = p0; i < p0 + sizeof(Pkt); ++i)
          if (ia_[i] != ib_[i])
            diverge(cyc, "backlog ring of sub-partition " + std::to_string(g) + " entry " + std::to_string(k) + " +" +
                             std::to_string(i - p0),
                    ia_[i], ib_[i]);
      }
    }
    // MALL lines: all of them are state
    const size_t mall0 = off + h.ovf * sizeof(Pkt);
    for (size_t i = mall0; i < mall0 + h.mall * sizeof(L2Line); ++i)
      if (ia_[i] != ib_[i])
        diverge(cyc, "MALL line " + std::to_string((i - mall0) / sizeof(L2Line)) + " +" +
                         std::to_string((i - mall0) % sizeof(L2Line)),
                ia_[i], ib_[i]);
  }
  [[noreturn]] void diverge(uint64_t cyc, const std::string& where, uint8_t va, uint8_t vb) {
    fail(cyc, "states diverge in " + where + " (" + a_->name() + " 0x" + hex(va) + ", " + b_->name() + " 0x" + hex(vb) + ")");
  }
  static std::string hex(uint8_t v) {
    char b[4];
    snprintf(b, sizeof(b), "%02x", v);
    return b;
  }
  [[noreturn]] void fail(uint64_t cyc, const std::string& what) {
    throw std::runtime_error("engine check failed at cycle " + std::to_string(cyc) + " (check point " +
                             std::to_string(checks_) + "): " + what);
  }

  std::unique_ptr<Engine> a_, b_;
  uint64_t every_, corrupt_at_;
  bool corrupt_mailbox_ = false;
  uint64_t checks_ = 0;
  uint32_t n_sm_ = 0, n_mem_ = 0, n_sub_per_mem_ = 1;
  std::vector<uint8_t> ia_, ib_;
};

}  // namespace

std::unique_ptr<Engine> make_check_engine(std::unique_ptr<Engine> primary, std::unique_ptr<Engine> reference,
                                          uint64_t interval, uint64_t corrupt_at, bool corrupt_mailbox) {
  return std::unique_ptr<Engine>(
      new CheckEngine(std::move(primary), std::move(reference), interval, corrupt_at, corrupt_mailbox));
}

}  // namespace asim
