// Epoch-synchronous (conservative PDES) driver logic shared by both engines.
//
// The reference advances every component in one serial loop per cycle
// (gpgpu_sim::cycle, gpu-sim.cc:1871-2107).  Here SMs and memory channels only
// interact through the interconnect, whose latency L (core cycles) is the
// lookahead: an epoch is L core cycles, packets injected in epoch e become
// visible at their destination in epoch e+1, so every SM and every channel
// can simulate a whole epoch independently (one wavefront each on the GPU)
// with ONE grid-wide barrier per epoch.  All cross-component decisions (CTA
// dispatch, kernel completion, idle fast-forward, deadlock) are computed
// redundantly and deterministically by every participant from state
// published at the previous epoch boundary -- no atomics, no races, and the
// CPU engine gives bit-identical results.
#pragma once
#include "mem.h"

namespace asim {

constexpr int kMaxChTot = 128;

// one unit's epoch-boundary publication: one 32-byte record, written by one
// store and read by one load per unit (the decision pass reads every unit)
struct UnitPub {
  uint64_t next;     // next-event time (fs, ~0 = none) for whole-epoch fast-forward:
                     // the first instant the unit can change state, or one of the
                     // packets it injected this epoch arrives (-sim_event_skip)
  uint64_t prog;     // SM: last progress cycle
  uint64_t insn;     // SM: thread instructions issued so far (-gpgpu_max_insn)
  uint32_t req;      // SM: CTA slots it can accept next epoch
  uint32_t idle;     // SM: drained and kernel fully dispatched; channel: idle
  uint32_t drained;  // SM: holds no work (launch latency may be pending)
  uint32_t ctas;     // SM: CTAs completed so far (-gpgpu_max_completed_cta)
  uint64_t pad;
};
static_assert(sizeof(UnitPub) == 48, "UnitPub layout");
// epoch-boundary publications, double buffered by epoch parity
struct EpochPub {
  UnitPub sm[2][kMaxSmTot];
  UnitPub ch[2][kMaxChTot];
  uint32_t next_cta[2];  // replicated dispatch cursor (published by SM 0)
  uint32_t pad[2];
};

// upper bound of one SM's quiet-cycle look-ahead at an epoch boundary
constexpr uint64_t kSkipHorizon = 1ull << 16;

// decision every participant derives after the barrier
struct EpochDecision {
  uint32_t done;        // kernel complete (all SMs idle)
  uint32_t all_idle;    // SMs and memory idle
  uint32_t deadlock;
  uint32_t limit;       // -gpgpu_max_insn / _max_completed_cta / _max_cta reached: stop
  uint64_t next_start;  // start cycle of the next epoch (after fast-forward)
};

// ---------------------------------------------------------------------------
// CTA dispatch: round-robin rounds over requesting SMs, rotated by epoch.
template <class P>
SIM_HDI void cta_dispatch(SMState& s, const SmCtx& x, SmKernel& ks, const UnitPub* pubs, uint32_t n_sm,
                          uint32_t rot) {
  const KernelDesc& k = *x.k;
  if (ks.next_cta >= k.n_cta) return;
  const uint32_t me = s.id;
  auto req = [&](int j) -> uint32_t { return pubs[j].req; };
  const uint32_t my_q = req((int)me);
  const uint32_t my_rank = (me + n_sm - rot) % n_sm;
  uint32_t base = ks.next_cta;
  for (uint32_t r = 0; r < (uint32_t)kMaxCta && base < k.n_cta; ++r) {
    uint32_t pr = P::sum((int)n_sm, [&](int j) -> uint32_t { return req(j) > r ? 1u : 0u; });
    if (pr == 0) break;
    if (my_q > r) {
      uint32_t pos = P::sum((int)n_sm, [&](int j) -> uint32_t {
        return (req(j) > r && ((uint32_t)j + n_sm - rot) % n_sm < my_rank) ? 1u : 0u;
      });
      uint32_t cta = base + pos;
      if (cta < k.n_cta) {
        // lowest free slot
        int slot = -1;
        for (uint32_t i = 0; i < s.kernel_cta_slots; ++i)
          if (!s.cta_valid[i]) { slot = (int)i; break; }
        if (slot >= 0) sm_launch_cta<P>(s, x, (uint32_t)slot, cta);
      }
    }
    base += pr;
  }
  ks.next_cta = base < k.n_cta ? base : k.n_cta;
}

SIM_HDI uint32_t sm_free_slots(const SMState& s) {
  return s.kernel_cta_slots > s.n_cta_active ? s.kernel_cta_slots - s.n_cta_active : 0;
}

// kernel (re)initialisation of an SM: first epoch of a new kernel
template <class P>
SIM_HDI void sm_kernel_init(SMState& s, const SmCtx& x, SmKernel& ks, uint64_t start, uint32_t flush_l1) {
  const KernelDesc& k = *x.k;
  ks.uid = k.uid;
  ks.next_cta = 0;
  ks.start_cycle = start;
  ks.ready_cycle = start + x.cfg->kernel_launch_latency + (uint64_t)x.cfg->tb_launch_latency * k.n_cta;
  s.kernel_cta_slots = k.cta_per_sm;
  if (flush_l1) {
    P::each(kMaxL1Lines, [&](int i) {
      s.l1[i].valid = 0;
      s.l1[i].dirty = 0;
    });
    P::sync();
  }
}

// one epoch of one SM: [t0, t1) core cycles
template <class P>
SIM_HDI void sm_epoch(SMState& s, const SmCtx& x, SmKernel& ks, const EpochPub& pub, uint32_t prev,
                      uint64_t t0, uint64_t t1, const Pkt* inbox, const uint32_t* incnt, uint32_t in_cap,
                      uint32_t n_sub, uint64_t epoch_idx) {
  const SimCfg& c = *x.cfg;
  // 0. cycles [s.cycle, t0) were fast-forwarded by epoch_decide (nothing could
  //    happen in them): account them exactly like quiet cycles
  if (t0 > s.cycle && (s.n_cta_active || !sm_idle(s))) sm_skip<P>(s, c, t0 - s.cycle);
  s.min_emit = ~0ull;
  // 1. arrivals (replies injected by the memory side last epoch)
  P::prof(12);
  gather_sorted<P>(inbox, incnt, s.id, n_sub, in_cap, t0 * c.per_core, s.inq, kInQ, s.inq_head, s.inq_n,
                   s_scratch_key(s), s_scratch_ref(s), s_scratch_rank(s), kInQ);
  // 2. CTA dispatch (state published at the previous boundary)
  P::prof(13);
  if (t0 >= ks.ready_cycle)
    // rotation by simulated time (t0 / epoch length), not by the epoch counter,
    // so fast-forwarded epochs leave the CTA -> SM assignment unchanged
    cta_dispatch<P>(s, x, ks, pub.sm[prev], c.n_sm, (uint32_t)((t0 / c.icnt_latency) % c.n_sm));
  // 3. (instructions are read from the kernel trace directly)
  P::prof(14);
  // 4. cycles
  P::prof(15);
  s.epoch_end = t1;
  if (P::uni(s.n_cta_active) || !sm_idle(s)) {
    P::tick(19);
    P::view(s, [&](auto& v) {
      for (uint64_t t = t0; t < t1;) {
        P::tick(17);
        sm_cycle<P>(v, x, t);
        ++t;
        if (t < t1 && c.event_skip) {
          // fast-forward cycles in which provably nothing happens
          P::tick(18);
          const uint64_t nx = P::uni(sm_quiet_until<P>(v, c, x.k->insts, t, t1));
          if (nx > t) {
            sm_skip<P>(v, c, nx - t);
            t = nx;
          }
        }
      }
    });
  }
  s.cycle = t1;
  P::prof(16);
}

// publish SM outbox counts + boundary state
template <class P>
SIM_HDI void sm_publish(SMState& s, const SmCtx& x, const SmKernel& ks, EpochPub& pub, uint32_t cur) {
  const SimCfg& c = *x.cfg;
  P::each((int)c.n_subpart, [&](int d) {
    x.outcnt[(uint64_t)d * x.n_src_sm + s.id] = s.ocnt[d];
    s.ocnt[d] = 0;
  });
  P::sync();
  const bool ready_for_cta = ks.next_cta < x.k->n_cta;
  const uint32_t req = ready_for_cta ? sm_free_slots(s) : 0u;
  const uint32_t idle = (ks.next_cta >= x.k->n_cta && sm_idle(s)) ? 1u : 0u;
  uint64_t nx = ~0ull;
  if (c.event_skip && (s.n_cta_active || !sm_idle(s)))
    nx = sm_quiet_until<P>(s, c, x.k->insts, s.cycle, s.cycle + kSkipHorizon) * c.per_core;
  nx = amin(nx, s.min_emit);
  UnitPub u;
  u.next = nx;
  u.prog = s.last_progress;
  u.insn = s.sget(SK(thread_insn));
  u.req = req;
  u.idle = idle;
  u.drained = sm_idle(s) ? 1u : 0u;
  u.ctas = (uint32_t)s.sget(SK(ctas_done));
  u.pad = 0;
  P::one([&] {
    pub.sm[cur][s.id] = u;
    if (s.id == 0) pub.next_cta[cur] = ks.next_cta;
  });
}

// one epoch of one memory channel
template <class P>
SIM_HDI void chan_epoch(ChanState& ch, const MemCtx& x, const Pkt* inbox, const uint32_t* incnt,
                        uint32_t in_cap, uint64_t t0_fs) {
  P::prof(20);
  ch.min_emit = ~0ull;
  mem_gather<P>(ch, *x.cfg, x, inbox, incnt, in_cap, t0_fs);
  P::one([&] {
    for (uint32_t j = 0; j < x.cfg->n_sub_per_mem; ++j) ch.sp[j].st.icnt_backlog += ch.sp[j].ovf_n;
  });
  P::prof(24);
  mem_window<P>(ch, x);
  P::prof(25);
}

template <class P>
SIM_HDI void chan_publish(ChanState& ch, const MemCtx& x, EpochPub& pub, uint32_t cur) {
  mem_publish<P>(ch, *x.cfg, x.outcnt);
  uint32_t idle = chan_idle(ch, *x.cfg) ? 1u : 0u;
  uint64_t nx = ~0ull;
  if (x.cfg->event_skip) nx = chan_next_event(ch, *x.cfg, amin(ch.t_dram, amin(ch.t_l2, ch.t_icnt)));
  nx = amin(nx, ch.min_emit);
  UnitPub u;
  u.next = nx;
  u.prog = 0;
  u.insn = 0;
  u.req = 0;
  u.idle = idle;
  u.drained = idle;
  u.ctas = 0;
  u.pad = 0;
  P::one([&] { pub.ch[cur][ch.id] = u; });
}

// every participant computes the same decision from the published state
template <class P>
SIM_HDI EpochDecision epoch_decide(const SimCfg& c, const EpochPub& pub, uint32_t cur, uint64_t t1,
                                   uint64_t ready_cycle, uint32_t next_cta_done, uint64_t epoch_idx,
                                   uint64_t max_cycle, uint32_t stop_when_issued = 0) {
  EpochDecision d;
  // one pass over every unit's record (one load per unit), then reductions
  uint32_t nbusy = 0, undrained = 0, nreq = 0, cbusy = 0, ctas = 0;
  uint64_t sm_next = ~0ull, ch_next = ~0ull, prog = 0, insn = 0;
  P::lane_loop((int)c.n_sm, [&](int j) {
    const UnitPub u = pub.sm[cur][j];
    insn += u.insn;
    ctas += u.ctas;
    nbusy += u.idle ? 0u : 1u;
    undrained += u.drained ? 0u : 1u;
    nreq += u.req ? 1u : 0u;
    sm_next = amin<uint64_t>(sm_next, u.next);
    prog = amax<uint64_t>(prog, u.prog & ((1ull << 56) - 1));  // progress stamps are < 2^56
  });
  P::lane_loop((int)c.n_mem, [&](int j) {
    const UnitPub u = pub.ch[cur][j];
    cbusy += u.idle ? 0u : 1u;
    ch_next = amin<uint64_t>(ch_next, u.next);
  });
  nbusy = P::uni(P::red_sum(nbusy));
  undrained = P::uni(P::red_sum(undrained));
  nreq = P::uni(P::red_sum(nreq));
  cbusy = P::uni(P::red_sum(cbusy));
  sm_next = P::uni(P::red_min64(sm_next));
  ch_next = P::uni(P::red_min64(ch_next));
  prog = P::uni(P::red_max64(prog));
  d.done = (nbusy == 0) ? 1u : 0u;
  d.all_idle = (nbusy == 0 && cbusy == 0) ? 1u : 0u;
  d.next_start = t1;
  d.deadlock = 0;
  // run caps checked while the kernel runs (reference gpgpu_sim::active,
  // gpu-sim.cc:1071-1094): instructions, completed CTAs, issued CTAs
  d.limit = 0;
  if (c.max_insn && P::uni(P::red_sum64(insn)) >= c.max_insn) d.limit = 1;
  if (c.max_completed_cta && P::uni(P::red_sum(ctas)) >= c.max_completed_cta) d.limit = 1;
  if (stop_when_issued && next_cta_done) d.limit = 1;
  // fast-forward over the kernel launch latency when nothing is in flight
  if (!next_cta_done && cbusy == 0 && t1 < ready_cycle && undrained == 0) {
    uint64_t E = c.icnt_latency;
    uint64_t skip = (ready_cycle - t1) / E * E;
    d.next_start = t1 + skip;
  }
  // Whole-epoch fast-forward (conservative PDES with exact next-event times):
  // the earliest instant any SM or channel can change state, any packet in
  // flight arrives, or the next CTA can be dispatched bounds how far every
  // participant can jump; epochs wholly before it are skipped.  With no
  // pending event at all (a deadlock) nothing is skipped.
  if (c.event_skip && !d.done) {
    uint64_t ev = amin(sm_next, ch_next);
    if (!next_cta_done && nreq) ev = amin(ev, amax(t1, ready_cycle) * c.per_core);
    if (ev != ~0ull) {
      const uint64_t E = c.icnt_latency;
      const uint64_t tc = ev / c.per_core;  // the next epoch may start no later than this
      if (tc >= t1 + E) {
        uint64_t s = t1 + (tc - t1) / E * E;
        if (max_cycle && s > max_cycle) s = max_cycle > t1 ? t1 + (max_cycle - t1 + E - 1) / E * E : t1;
        if (s > d.next_start) d.next_start = s;
      }
    }
  }
  if (c.deadlock_window && nbusy && ((t1 / c.icnt_latency) & 63) == 0) {
    // newest progress stamp over all SMs
    const uint64_t last = prog;
    if (t1 > last + c.deadlock_window && t1 > ready_cycle + c.deadlock_window) d.deadlock = 1;
  }
  return d;
}

}  // namespace asim
