// CPU reference engine: the cycle model with the sequential lane policy.
// SMs / channels of one epoch are independent (PDES), so the epoch body runs
// on a persistent thread team (thread_team.h, -sim_cpu_threads); results are
// bit-identical for any thread count.
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include <functional>

#include <atomic>
#include <exception>
#include <mutex>

#include "engine.h"
#include "thread_team.h"
#include "trace_window.h"

namespace asim {

uint32_t reply_cap(const SimCfg& c) {
  // icnt ticks per epoch, +1 for phase alignment (at the slowest core clock
  // DVFS may choose: an epoch is icnt_latency core cycles)
  uint64_t win = (uint64_t)c.icnt_latency * std::max(c.per_core, c.per_core_max);
  return (uint32_t)((win + c.per_icnt - 1) / c.per_icnt + 1);
}

void check_core_clock(const SimCfg& c, uint64_t per_core) {
  if (per_core == 0 || per_core > std::max(c.per_core, c.per_core_max))
    throw std::runtime_error("set_core_clock: core period beyond the configured DVFS range (-dvfs_min_clock_ratio)");
}

void init_sm_state(SMState& s, uint32_t id) {
  memset(&s, 0, sizeof(SMState));
  s.id = id;
}

void init_chan_state(ChanState& ch, uint32_t id, const SimCfg& c) {
  memset(&ch, 0, sizeof(ChanState));
  ch.id = id;
  ch.t_icnt = 0;
  ch.t_l2 = 0;
  ch.t_dram = 0;
  (void)c;
}

void host_memcpy_fill(ChanState* chs, uint32_t nch, const SimCfg& c, uint64_t addr, uint64_t bytes) {
  // with XCD-private L2s a host copy (SDMA) lands in memory, not in any XCD's L2
  if (c.l2.disabled || c.n_xcd) return;
  const uint64_t first = addr & ~127ull;
  const uint64_t last = (addr + bytes + 127) & ~127ull;
  // only the tail that can still be resident matters
  uint64_t cap_lines = (uint64_t)c.l2.nsets * c.l2.assoc * c.n_subpart;
  uint64_t start = first;
  if ((last - first) / 128 > 2 * cap_lines) start = last - 2 * cap_lines * 128;
  for (uint64_t line = start; line < last; line += 128) {
    AddrTlx t = addr_decode(c, line);
    uint32_t ch = t.sub / c.n_sub_per_mem, sub = t.sub % c.n_sub_per_mem;
    if (ch >= nch) continue;
    SubPart& sp = chs[ch].sp[sub];
    L2Line* T = l2_tags(chs[ch], c, sub);
    uint32_t set = l2_set(c, line);
    int way = l2_find<SeqPar>(T, c.l2, set, line);
    if (way < 0) {
      way = l2_victim<SeqPar>(T, c.l2, set);
      L2Line& L = T[set * c.l2.assoc + way];
      L.tag = line;
      L.dirty = 0;
      L.valid = 0;
    }
    L2Line& L = T[set * c.l2.assoc + way];
    uint64_t lo = std::max(line, addr), hi = std::min(line + 128, addr + bytes);
    for (uint64_t s = (lo - line) >> 5; s <= ((hi - 1 - line) >> 5) && s < 4; ++s) L.valid |= (uint8_t)(1u << s);
    L.lru = ++sp.l2_stamp;
  }
}

void check_state_header(const EngineStateHeader& h, const EngineStateHeader& w) {
  if (h.magic != w.magic || h.version != w.version) throw std::runtime_error("engine state: not a state image");
  if (h.n_sm != w.n_sm || h.n_mem != w.n_mem || h.sm_bytes != w.sm_bytes || h.ch_bytes != w.ch_bytes ||
      h.pub_bytes != w.pub_bytes || h.box_req != w.box_req || h.cnt_req != w.cnt_req || h.box_rep != w.box_rep ||
      h.cnt_rep != w.cnt_rep || h.ovf != w.ovf || h.mall != w.mall || h.links != w.links)
    throw std::runtime_error("engine state: image was written for a different configuration or build");
}

void host_flush_l2(ChanState* chs, uint32_t nch, const SimCfg& c, bool writeback, L2Line* mall) {
  const uint32_t per_sub = c.l2.nsets * c.l2.assoc;
  for (uint32_t i = 0; i < nch; ++i) {
    ChanState& ch = chs[i];
    if (writeback && !c.l2.disabled) {
      // sub-partition by sub-partition, lines in index order: the same order
      // on every engine, so the MALL contents stay bit-exact
      for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
        MemStats& st = ch.sp[j].st;
        const L2Line* T = l2_tags(ch, c, j);
        for (uint32_t k = 0; k < per_sub; ++k) {
          const L2Line& L = T[k];
          if (!(L.valid && L.dirty)) continue;
          const uint32_t n = (uint32_t)popc64(L.dirty);
          st.l2_mem_wr += n;
          st.l2_mem_wr_req += wr_requests(L.dirty);
          st.l2_evict_dirty++;
          if (!mall) {
            st.dram_wr += n;  // straight to DRAM, untimed (between kernels)
            continue;
          }
          L2Line* b = mall + (size_t)i * mall_lines(c) + (size_t)mall_set(c, L.tag) * c.mall_assoc;
          int w = mall_find<SeqPar>(b, c.mall_assoc, L.tag);
          if (w < 0) {
            w = mall_victim<SeqPar>(b, c.mall_assoc);
            if (b[w].valid && b[w].dirty) {
              const uint32_t nv = (uint32_t)popc64(b[w].dirty);
              ch.sp[0].st.mall_wb += nv;
              ch.sp[0].st.dram_wr += nv;
            }
            b[w] = L2Line{};
            b[w].tag = L.tag;
          }
          b[w].valid |= L.dirty;
          b[w].dirty |= L.dirty;
          b[w].lru = ++ch.mall_stamp;
          ch.sp[0].st.mall_wr += n;
        }
      }
    }
    for (auto& L : ch.l2) {
      L.valid = 0;
      L.dirty = 0;
    }
  }
}

namespace {

class CpuEngine : public Engine {
 public:
  const char* name() const override { return "cpu"; }

  void init(const SimCfg& c) override {
    c_ = c;
    sms_.assign(c.n_sm, SMState());
    for (uint32_t i = 0; i < c.n_sm; ++i) init_sm_state(sms_[i], i);
    chs_.assign(c.n_mem, ChanState());
    for (uint32_t i = 0; i < c.n_mem; ++i) init_chan_state(chs_[i], i, c);
    pub_.reset(new EpochPub());
    memset(pub_.get(), 0, sizeof(EpochPub));
    cap_req_ = c.icnt_latency;
    cap_rep_ = reply_cap(c);
    for (int p = 0; p < 2; ++p) {
      box_req_[p].assign((size_t)c.n_subpart * c.n_sm * cap_req_, Pkt{});
      cnt_req_[p].assign((size_t)c.n_subpart * c.n_sm, 0);
      box_rep_[p].assign((size_t)c.n_sm * c.n_subpart * cap_rep_, Pkt{});
      cnt_rep_[p].assign((size_t)c.n_sm * c.n_subpart, 0);
    }
    ovf_cap_ = backlog_cap(c);
    ovf_.assign((size_t)c.n_subpart * ovf_cap_, Pkt{});
    mall_.assign((size_t)(c.n_mem * mall_lines(c)), L2Line{});
    link_free_.clear();
    link_refs_.clear();
    n_link_state_ = 0;
    if (c.link_contention && (icnt_link_count(c) > kMaxIcntLinks || !icnt_contention_fits(c, cap_req_, cap_rep_) ||
                              icnt_scratch_words(c, cap_req_, cap_rep_) > kMaxIcntScratchWords))
      throw std::runtime_error("-icnt_link_contention: topology or mailboxes too large for the link pass");
    if (icnt_contention_on(c)) {
      // the link model's persistent words, then its two statistics words
      n_link_state_ = (size_t)icnt_state_words(c, cap_req_, cap_rep_);
      link_free_.assign(n_link_state_ + kIcntStatWords, 0);
      link_refs_.assign((size_t)icnt_scratch_words(c, cap_req_, cap_rep_), 0);
    }
    epoch_ = 0;
    cycle_ = 0;
    kt_ = KernelTab{};
    kt_.mix = c.concurrent_kernel_sm;
    if (c_.trace_mask) {
      const size_t units = (size_t)c.n_sm + c.n_mem;
      trace_ev_.assign(units * c_.trace_cap, TraceEv{});
      trace_cnt_.assign(units, 0);
      c_.trace_ev = trace_ev_.data();
      c_.trace_cnt = trace_cnt_.data();
    }
  }

  void trace_drain(std::vector<TraceEv>& out, uint64_t* dropped) override {
    out.clear();
    for (size_t u = 0; u < trace_cnt_.size(); ++u) {
      const uint32_t n = trace_cnt_[u], k = std::min(n, c_.trace_cap);
      out.insert(out.end(), trace_ev_.begin() + (long)(u * c_.trace_cap), trace_ev_.begin() + (long)(u * c_.trace_cap + k));
      if (dropped) *dropped += n - k;
      trace_cnt_[u] = 0;
    }
  }

  void launch(uint32_t slot, ReadyKernel& k, const KernelDesc& kd) override {
    if (slot >= (uint32_t)kMaxConc || (kt_.active >> slot & 1u)) throw std::runtime_error("launch: kernel slot busy");
    if (!k.streamed() && k.insts.size() > kIdxMask) throw std::runtime_error("kernel trace exceeds 2^29 warp instructions");
    KernelDesc& d = kt_.k[slot];
    d = kd;
    // the whole trace in place, or (host-streamed trace) rings of a window
    // of CTAs that follows the dispatch cursor (trace_window.h)
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
    // serial, or a persistent team (thread_team.h): every thread runs the
    // same epoch loop over an interleaved share of the units, one barrier
    // per epoch, and evaluates the epoch decision itself (it is a pure
    // function of the published state), so they all stop at the same epoch
    const uint32_t nthr = std::max<uint32_t>(1, std::min<uint32_t>(c_.cpu_threads, (uint32_t)(sms_.size() + chs_.size())));
    bar_.reset(nthr);
    const uint64_t epoch0 = epoch_, cycle0 = cycle_;
    uint64_t end_epoch = epoch0, end_cycle = cycle0;
    // a throw inside the team (a malformed streamed trace in tw_.ensure, a
    // CTA-fit logic error, ...) must not leave the other threads spinning at
    // a barrier the thrower never reaches: the thread records the first
    // exception and still arrives at the next barrier, after which every
    // thread sees the abort flag and leaves the loop; run() rethrows once the
    // whole team has returned
    std::atomic<bool> abort{false};
    std::exception_ptr err;
    std::mutex err_mu;
    auto fail = [&]() {
      std::lock_guard<std::mutex> g(err_mu);
      if (!err) err = std::current_exception();
      abort.store(true, std::memory_order_release);
    };
    std::function<void(uint32_t)> job = [&](uint32_t tid) {
      const SimCfg& c = c_;
      const uint64_t E = c.icnt_latency;
      const int nsm = (int)sms_.size(), nch = (int)chs_.size();
      uint64_t epoch = epoch0, cycle = cycle0, epochs = 0;
      bool refill = true;
      // armed power sampler: the next sample point (every thread tracks it)
      uint64_t pw_next = pw_on_ ? pw_.t_prev + pw_.freq : 0;
      // destinations with packets in the previous epoch's mailboxes (all at a
      // run's first epoch): the gathers of the others are skipped
      uint64_t reqm[2] = {~0ull, ~0ull}, repm[2] = {~0ull, ~0ull};
      RunResult r;
      for (;;) {
        // host-streamed traces: bring in the CTAs the next epochs can
        // dispatch (epoch_decide flags when the window falls short)
        if (refill && tw_.any_streamed()) {
          if (nthr > 1) bar_.wait();
          if (tid == 0) {
            try {
              tw_.ensure(kt_, c, [&](DispatchView& v) { read_dispatch(v); });
            } catch (...) {
              fail();
            }
          }
          if (nthr > 1) bar_.wait();
          if (abort.load(std::memory_order_acquire)) break;
        }
        const uint32_t cur = (uint32_t)(epoch & 1), prev = cur ^ 1u;
        const uint64_t t0 = cycle, t1 = t0 + E;
        // contiguous shares (SMs, then channels, each split evenly): a
        // thread's units' mailbox counters and published records share cache
        // lines with its own units, not with every other thread's
        const int s0 = (int)((uint64_t)nsm * tid / nthr), s1 = (int)((uint64_t)nsm * (tid + 1) / nthr);
        const int c0 = (int)((uint64_t)nch * tid / nthr), c1 = (int)((uint64_t)nch * (tid + 1) / nthr);
        try {
        for (int q = 0; q < (s1 - s0) + (c1 - c0); ++q) {
          const int i = q < s1 - s0 ? s0 + q : nsm + c0 + (q - (s1 - s0));
          if (i < nsm) {
            SMState& s = sms_[i];
            SmCtx x = ctx_sm(cur);
            sm_epoch<SeqPar>(s, x, *pub_, prev, t0, t1, box_rep_[prev].data(), cnt_rep_[prev].data(), cap_rep_,
                             c.n_subpart, epoch, repm);
            sm_publish<SeqPar>(s, x, *pub_, cur);
          } else {
            ChanState& ch = chs_[i - nsm];
            MemCtx m = ctx_mem(cur, t1);
            m.mall = mall_.empty() ? nullptr : mall_.data() + (size_t)(i - nsm) * mall_lines(c);
            chan_epoch<SeqPar>(ch, m, box_req_[prev].data(), cnt_req_[prev].data(), cap_req_, core_fs(c, t0), reqm);
            chan_publish<SeqPar>(ch, m, *pub_, cur);
          }
        }
        } catch (...) {
          fail();
        }
        if (nthr > 1) bar_.wait();
        if (abort.load(std::memory_order_acquire)) break;
        if (!link_free_.empty()) {
          // shared links of multi-hop routes: this epoch's packets reserve
          // their routes before any destination reads them (icnt_links.h)
          if (tid == 0) {
            try {
              icnt_epoch_pass<SeqPar>(c, box_req_[cur].data(), cnt_req_[cur].data(), cap_req_, box_rep_[cur].data(),
                                      cnt_rep_[cur].data(), cap_rep_, link_free_.data(), link_refs_.data());
            } catch (...) {
              fail();
            }
          }
          if (nthr > 1) bar_.wait();
          if (abort.load(std::memory_order_acquire)) break;
        }
        const uint64_t mc = pw_on_ ? (lim.max_cycle ? std::min(lim.max_cycle, pw_next) : pw_next) : lim.max_cycle;
        const EpochDecision d = epoch_decide<SeqPar>(c, *pub_, cur, t1, kt_, epoch, mc);
        refill = d.refill != 0;
        reqm[0] = d.req_dst[0];
        reqm[1] = d.req_dst[1];
        repm[0] = d.rep_dst[0];
        repm[1] = d.rep_dst[1];
        ++epoch;
        ++epochs;
        cycle = d.next_start;
        if (pw_on_) {
          const bool exits = d.done || d.deadlock || d.limit || (lim.max_cycle && cycle >= lim.max_cycle) ||
                             (lim.max_epochs && epochs >= lim.max_epochs);
          if (exits || cycle >= pw_next) {
            // thread 0 samples while the others wait (the next epoch would
            // move the statistics)
            if (tid == 0) {
              try {
                power_sample(cycle);
              } catch (...) {
                fail();
              }
            }
            if (nthr > 1) bar_.wait();
            if (abort.load(std::memory_order_acquire)) break;
            pw_next = cycle + pw_.freq;
          }
        }
        if (d.done) {
          r.done = true;
          r.done_mask = d.done;
        } else if (d.deadlock) {
          r.deadlock = true;
        } else if (d.limit) {
          r.hit_limit = true;
          r.cap = true;
        } else if ((lim.max_cycle && cycle >= lim.max_cycle) || (lim.max_epochs && epochs >= lim.max_epochs)) {
          r.hit_limit = true;
        } else {
          continue;
        }
        break;
      }
      if (tid == 0) {
        r.epochs = epochs;
        res = r;
        end_epoch = epoch;
        end_cycle = cycle;
      }
    };
    team_.run(nthr, job);
    if (err) std::rethrow_exception(err);
    epoch_ = end_epoch;
    cycle_ = end_cycle;
    if (res.done) {
      kt_.active &= ~res.done_mask;
      for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
        if (res.done_mask >> k & 1u) tw_.done(k);
    }
    res.end_cycle = cycle_;
    return res;
  }

  uint64_t now() const override { return cycle_; }
  void trace_residency(uint64_t* peak_bytes, uint64_t* refills) const override {
    *peak_bytes = tw_.resident_peak;
    *refills = tw_.refills;
  }
  bool power_sampler() const override { return true; }
  void power_arm(const PwrArm& a) override {
    pw_ = a;
    pw_on_ = true;
    pw_out_.clear();
  }
  void power_disarm() override { pw_on_ = false; }
  void power_drain(std::vector<PwrSample>& out) override {
    out.swap(pw_out_);
    pw_out_.clear();
  }
  void power_sample(uint64_t now) {
    std::vector<const MemStats*> mem;
    for (auto& ch : chs_)
      for (uint32_t j = 0; j < c_.n_sub_per_mem; ++j) mem.push_back(&ch.sp[j].st);
    std::vector<const SMStats*> sm(sms_.size());
    for (size_t i = 0; i < sms_.size(); ++i) sm[i] = &sms_[i].st;
    double S[PS_COUNT];
    pwr_sums_of(sm.data(), sm.size(), mem.data(), mem.size(), S);
    pw_out_.push_back(pwr_take(pw_, S, now));
  }
  void read_dispatch(DispatchView& v) const {
    const SMState& s0 = sms_[0];
    memcpy(v.k_uid, s0.k_uid, sizeof(v.k_uid));
    memcpy(v.next_cta, s0.next_cta, sizeof(v.next_cta));
    memcpy(v.next_ctax, s0.next_ctax, sizeof(v.next_ctax));
    v.sms.resize(sms_.size());
    for (size_t m = 0; m < sms_.size(); ++m) {
      memcpy(v.sms[m].cta_id, sms_[m].cta_id, sizeof(v.sms[m].cta_id));
      memcpy(v.sms[m].cta_valid, sms_[m].cta_valid, sizeof(v.sms[m].cta_valid));
      memcpy(v.sms[m].cta_ks, sms_[m].cta_ks, sizeof(v.sms[m].cta_ks));
    }
  }
  struct HostMem {
    static constexpr bool kHost = true;
    void* alloc(size_t n) { return std::malloc(n); }
    void free(void* p) { std::free(p); }
    void write(void* d, const void* h, size_t n) { memcpy(d, h, n); }
  };
  TraceWindows<HostMem> tw_;
  bool pw_on_ = false;
  PwrArm pw_;
  std::vector<PwrSample> pw_out_;
  ThreadTeam team_;
  SpinBarrier bar_;
  std::vector<TraceEv> trace_ev_;
  std::vector<uint32_t> trace_cnt_;

  void memcpy_fill_l2(uint64_t addr, uint64_t bytes) override {
    host_memcpy_fill(chs_.data(), (uint32_t)chs_.size(), c_, addr, bytes);
  }
  void set_core_clock(uint64_t per_core, uint64_t base_cyc, uint64_t base_fs) override {
    check_core_clock(c_, per_core);
    c_.per_core = per_core;
    c_.clk_base_cyc = base_cyc;
    c_.clk_base_fs = base_fs;
    cfg_set_divs(c_);
  }
  void flush_l2(bool writeback) override {
    host_flush_l2(chs_.data(), (uint32_t)chs_.size(), c_, writeback, mall_.empty() ? nullptr : mall_.data());
  }

  void stats(std::vector<SMStats>& sm, std::vector<MemStats>& mem) override {
    sm.clear();
    mem.clear();
    for (auto& s : sms_) sm.push_back(s.st);
    for (auto& ch : chs_)
      for (uint32_t j = 0; j < c_.n_sub_per_mem; ++j) mem.push_back(ch.sp[j].st);
  }

  void snapshot(std::vector<uint8_t>& out) override {
    out.resize(sms_.size() * sizeof(SMState) + chs_.size() * sizeof(ChanState) + mall_.size() * sizeof(L2Line) +
               n_link_state_ * 8);
    uint8_t* p = out.data();
    for (auto& s : sms_) {
      memcpy(p, &s, sizeof(SMState));
      p += sizeof(SMState);
    }
    for (auto& ch : chs_) {
      memcpy(p, &ch, sizeof(ChanState));
      p += sizeof(ChanState);
    }
    if (!mall_.empty()) memcpy(p, mall_.data(), mall_.size() * sizeof(L2Line));
    p += mall_.size() * sizeof(L2Line);
    if (n_link_state_) memcpy(p, link_free_.data(), n_link_state_ * 8);
  }
  void restore(const std::vector<uint8_t>& in) override {
    if (in.size() != sms_.size() * sizeof(SMState) + chs_.size() * sizeof(ChanState) + mall_.size() * sizeof(L2Line) +
                         n_link_state_ * 8)
      throw std::runtime_error("snapshot size mismatch");
    const uint8_t* p = in.data();
    for (auto& s : sms_) {
      memcpy(&s, p, sizeof(SMState));
      p += sizeof(SMState);
    }
    for (auto& ch : chs_) {
      memcpy(&ch, p, sizeof(ChanState));
      p += sizeof(ChanState);
    }
    if (!mall_.empty()) memcpy(mall_.data(), p, mall_.size() * sizeof(L2Line));
    p += mall_.size() * sizeof(L2Line);
    if (n_link_state_) memcpy(link_free_.data(), p, n_link_state_ * 8);
  }
  void link_stats(uint64_t* delayed, uint64_t* wait_cycles, uint64_t* deadlocked) override {
    *delayed = n_link_state_ ? link_free_[n_link_state_] : 0;
    *wait_cycles = n_link_state_ ? link_free_[n_link_state_ + 1] : 0;
    if (deadlocked) *deadlocked = n_link_state_ ? link_free_[n_link_state_ + 2] : 0;
  }
  void advance(uint64_t cycles) override {
    uint64_t E = c_.icnt_latency;
    cycle_ += (cycles + E - 1) / E * E;
  }

  EngineStateHeader header() const {
    EngineStateHeader h;
    h.n_sm = sms_.size();
    h.n_mem = chs_.size();
    h.sm_bytes = sizeof(SMState);
    h.ch_bytes = sizeof(ChanState);
    h.pub_bytes = sizeof(EpochPub);
    h.box_req = box_req_[0].size();
    h.cnt_req = cnt_req_[0].size();
    h.box_rep = box_rep_[0].size();
    h.cnt_rep = cnt_rep_[0].size();
    h.ovf = ovf_.size();
    h.mall = mall_.size();
    h.links = link_free_.size();
    h.cycle = cycle_;
    h.epoch = epoch_;
    h.ready = kt_.active;
    return h;
  }

  void save_state(std::vector<uint8_t>& out) override {
    out.clear();
    StateOut o{out};
    EngineStateHeader h = header();
    o.put(&h, sizeof(h));
    o.put(sms_.data(), sms_.size() * sizeof(SMState));
    o.put(chs_.data(), chs_.size() * sizeof(ChanState));
    o.put(pub_.get(), sizeof(EpochPub));
    for (int p = 0; p < 2; ++p) {
      o.put(box_req_[p].data(), box_req_[p].size() * sizeof(Pkt));
      o.put(cnt_req_[p].data(), cnt_req_[p].size() * sizeof(uint32_t));
      o.put(box_rep_[p].data(), box_rep_[p].size() * sizeof(Pkt));
      o.put(cnt_rep_[p].data(), cnt_rep_[p].size() * sizeof(uint32_t));
    }
    o.put(ovf_.data(), ovf_.size() * sizeof(Pkt));
    o.put(mall_.data(), mall_.size() * sizeof(L2Line));
    if (!link_free_.empty()) o.put(link_free_.data(), link_free_.size() * 8);
  }

  void load_state(const std::vector<uint8_t>& in) override {
    StateIn r{in};
    EngineStateHeader h;
    r.get(&h, sizeof(h));
    check_state_header(h, header());
    r.get(sms_.data(), sms_.size() * sizeof(SMState));
    r.get(chs_.data(), chs_.size() * sizeof(ChanState));
    r.get(pub_.get(), sizeof(EpochPub));
    for (int p = 0; p < 2; ++p) {
      r.get(box_req_[p].data(), box_req_[p].size() * sizeof(Pkt));
      r.get(cnt_req_[p].data(), cnt_req_[p].size() * sizeof(uint32_t));
      r.get(box_rep_[p].data(), box_rep_[p].size() * sizeof(Pkt));
      r.get(cnt_rep_[p].data(), cnt_rep_[p].size() * sizeof(uint32_t));
    }
    r.get(ovf_.data(), ovf_.size() * sizeof(Pkt));
    r.get(mall_.data(), mall_.size() * sizeof(L2Line));
    if (!link_free_.empty()) r.get(link_free_.data(), link_free_.size() * 8);
    cycle_ = h.cycle;
    epoch_ = h.epoch;
    if (h.ready) throw std::runtime_error("engine state: image taken with kernels running");
  }

 private:
  SmCtx ctx_sm(uint32_t cur) {
    SmCtx x;
    x.cfg = &c_;
    x.kt = &kt_;
    x.outbox = box_req_[cur].data();
    x.outcnt = cnt_req_[cur].data();
    x.out_cap = cap_req_;
    x.n_src_sm = c_.n_sm;
    x.rt_st = c_.link_contention == 2 && !link_free_.empty() ? link_free_.data() : nullptr;
    return x;
  }
  MemCtx ctx_mem(uint32_t cur, uint64_t t1) {
    MemCtx m;
    m.cfg = &c_;
    m.outbox = box_rep_[cur].data();
    m.outcnt = cnt_rep_[cur].data();
    m.out_cap = cap_rep_;
    m.n_src_sub = c_.n_subpart;
    m.win_end = core_fs(c_, t1);
    m.ovf = ovf_.data();
    m.ovf_cap = ovf_cap_;
    m.mall = nullptr;
    m.rt_st = c_.link_contention == 2 && !link_free_.empty() ? link_free_.data() : nullptr;
    return m;
  }

  SimCfg c_{};
  std::vector<SMState> sms_;
  std::vector<ChanState> chs_;
  std::unique_ptr<EpochPub> pub_;
  std::vector<Pkt> box_req_[2], box_rep_[2];
  std::vector<uint32_t> cnt_req_[2], cnt_rep_[2];
  uint32_t cap_req_ = 0, cap_rep_ = 0;
  std::vector<Pkt> ovf_;  // arrival backlog rings [n_subpart][ovf_cap_]
  std::vector<L2Line> mall_;  // MALL lines [n_mem][mall_sets * mall_assoc]
  uint32_t ovf_cap_ = 0;
  // -icnt_link_contention: the link model's persistent state (link free
  // times, or the router network's, icnt_router.h), then {delayed packets,
  // delay in interconnect cycles}; and the pass's scratch
  std::vector<uint64_t> link_free_;
  std::vector<uint32_t> link_refs_;
  size_t n_link_state_ = 0;
  uint64_t epoch_ = 0, cycle_ = 0;
  KernelTab kt_{};
};

}  // namespace

std::unique_ptr<Engine> make_cpu_engine() { return std::unique_ptr<Engine>(new CpuEngine()); }

}  // namespace asim
