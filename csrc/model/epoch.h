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
#include "icnt_router.h"
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
  uint32_t req;      // SM: bit k: it requests CTAs of the kernel in slot k next epoch
  uint16_t idle;     // SM: drained and every kernel fully dispatched; channel: idle
  uint8_t kbusy;     // SM: bit k: it holds CTAs of the kernel in slot k
  uint8_t pad8;
  uint32_t drained;  // SM: holds no work (launch latency may be pending)
  uint32_t ctas;     // SM: CTAs completed so far (-gpgpu_max_completed_cta)
  uint64_t reqk;     // SM: byte k: CTAs of slot k it can accept next epoch
  uint64_t dmask[2]; // destinations it put packets for this epoch (bit d % 128; SM: sub-partitions, channel: SMs)
};
static_assert(sizeof(UnitPub) == 64, "UnitPub layout");
// epoch-boundary publications, double buffered by epoch parity
struct EpochPub {
  UnitPub sm[2][kMaxSmTot];
  UnitPub ch[2][kMaxChTot];
  uint32_t next_cta[2][kMaxConc];  // replicated dispatch cursors per kernel slot (published by SM 0)
  uint32_t next_ctax[2][kMaxConc][kMaxXcd];  // -sim_xcd: the per-XCD cursors behind next_cta
};

// upper bound of one SM's quiet-cycle look-ahead at an epoch boundary
constexpr uint64_t kSkipHorizon = 1ull << 16;

// decision every participant derives after the barrier
struct EpochDecision {
  uint32_t done;        // bit k: the kernel in slot k completed
  uint32_t all_idle;    // SMs and memory idle
  uint32_t deadlock;
  uint32_t limit;       // -gpgpu_max_insn / _max_completed_cta / _max_cta reached: stop
  uint32_t refill;      // the next epoch's dispatch could need a CTA whose trace is not resident
  uint64_t next_start;  // start cycle of the next epoch (after fast-forward)
  // destinations (bit d % 128) that have packets in this epoch's mailboxes:
  // the next epoch's gathers skip the others (their cells are all zero)
  uint64_t req_dst[2];  // sub-partitions with requests
  uint64_t rep_dst[2];  // SMs with replies
};

// ---------------------------------------------------------------------------
// CTA dispatch (reference gpgpu_sim::issue_block2core, gpu-sim.cc and
// simt_core_cluster::issue_block2core, shader.cc:4502-4535): round-robin
// rounds over the SMs requesting CTAs of one kernel, rotated by epoch.
template <class P, class S>
SIM_HDI void cta_dispatch(S& s, const SmCtx& x, uint32_t ks, const UnitPub* pubs, uint32_t n_sm,
                          uint32_t rot) {
  const KernelDesc& k = x.kt->k[ks];
  if (s.next_cta[ks] >= k.n_cta) return;
  const uint32_t me = s.id;
  const uint32_t sh = ks * 8;
  auto req = [&](int j) -> uint32_t { return (uint32_t)(pubs[j].reqk >> sh) & 0xffu; };
  const uint32_t my_q = req((int)me);
  const uint32_t my_rank = (me + n_sm - rot) % n_sm;
  uint32_t base = s.next_cta[ks];
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
        for (uint32_t i = 0; i < (uint32_t)kMaxCta; ++i)
          if (!s.cta_valid[i]) { slot = (int)i; break; }
        if (slot >= 0) sm_launch_cta<P>(s, x, (uint32_t)slot, cta, ks);
      }
    }
    base += pr;
  }
  s.next_cta[ks] = base < k.n_cta ? base : k.n_cta;
}

// -sim_xcd: the hardware hands workgroup i to XCD i % n_xcd (round robin
// over the XCDs at every dispatch), so the CTAs of residue x go to the SMs of
// XCD x (SM s belongs to XCD s % n_xcd), in the same rounds as above within
// each XCD.  Every SM advances every XCD's cursor (the state is replicated).
template <class P, class S>
SIM_HDI void cta_dispatch_xcd(S& s, const SmCtx& x, uint32_t ks, const UnitPub* pubs, uint32_t n_sm,
                              uint32_t rot) {
  const KernelDesc& k = x.kt->k[ks];
  if (s.next_cta[ks] >= k.n_cta) return;
  const uint32_t nx = x.cfg->n_xcd;
  const uint32_t me = s.id;
  const uint32_t sh = ks * 8;
  auto req = [&](int j) -> uint32_t { return (uint32_t)(pubs[j].reqk >> sh) & 0xffu; };
  const uint32_t my_q = req((int)me);
  const uint32_t my_rank = (me + n_sm - rot) % n_sm;
  uint32_t total = 0;
  for (uint32_t xi = 0; xi < nx; ++xi) {
    const uint32_t ncx = k.n_cta > xi ? (k.n_cta - xi + nx - 1) / nx : 0u;
    uint32_t base = s.next_ctax[ks][xi];
    for (uint32_t r = 0; r < (uint32_t)kMaxCta && base < ncx; ++r) {
      const uint32_t pr = P::sum((int)n_sm, [&](int j) -> uint32_t {
        return ((uint32_t)j % nx == xi && req(j) > r) ? 1u : 0u;
      });
      if (pr == 0) break;
      if (me % nx == xi && my_q > r) {
        const uint32_t pos = P::sum((int)n_sm, [&](int j) -> uint32_t {
          return ((uint32_t)j % nx == xi && req(j) > r && ((uint32_t)j + n_sm - rot) % n_sm < my_rank) ? 1u : 0u;
        });
        const uint32_t j = base + pos;
        if (j < ncx) {
          int slot = -1;
          for (uint32_t i = 0; i < (uint32_t)kMaxCta; ++i)
            if (!s.cta_valid[i]) { slot = (int)i; break; }
          if (slot >= 0) sm_launch_cta<P>(s, x, (uint32_t)slot, xi + nx * j, ks);
        }
      }
      base += pr;
    }
    s.next_ctax[ks][xi] = base < ncx ? base : ncx;
    total += s.next_ctax[ks][xi];
  }
  s.next_cta[ks] = total;
}

// Highest CTA id the next epoch's dispatch can hand out (an upper bound: every
// SM takes at most cta_per_sm CTAs per epoch; with -sim_xcd CTA xi + nx * j
// comes from XCD xi's cursor j).  The GPU engine keeps the traces of CTAs up
// to this bound resident (-gpu_trace_window); host and device use this one
// formula.
SIM_HDI uint64_t dispatch_bound(const SimCfg& c, const KernelDesc& k, uint32_t next, const uint32_t* nextx) {
  const uint64_t cpc = amin<uint32_t>(k.cta_per_sm, kMaxCta);
  if (c.n_xcd > 1) {
    const uint64_t nx = c.n_xcd;
    uint32_t mb = 0;
    for (uint32_t xi = 0; xi < c.n_xcd; ++xi) mb = amax<uint32_t>(mb, nextx[xi]);
    return (nx - 1) + nx * ((uint64_t)mb + (c.n_sm + nx - 1) / nx * cpc);
  }
  return (uint64_t)next + (uint64_t)c.n_sm * cpc;
}

// kernel slots in launch (uid) order: older kernels are served first
SIM_HDI uint32_t slot_order(const KernelTab& kt, uint8_t* order) {
  uint32_t n = 0;
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k) {
    if (!(kt.active >> k & 1u)) continue;
    uint32_t i = n++;
    while (i > 0 && kt.k[order[i - 1]].uid > kt.k[k].uid) {
      order[i] = order[i - 1];
      --i;
    }
    order[i] = (uint8_t)k;
  }
  return n;
}

// CTAs of kernel slot `ks` this SM can accept on top of what it holds and of
// `held` warps / `thr` threads / ... already promised to older kernels
// (shader_core_ctx::can_issue_1block / occupy_shader_resource_1block):
// per-kernel CTA limit, CTA slots, threads, registers, shared memory, and a
// contiguous run of free warps per CTA
struct SmRes {
  uint64_t wmask;
  uint32_t ctas, thr, regs, shmem;
};
template <class S>
SIM_HDI uint32_t sm_cta_fit(const S& s, const SimCfg& c, const KernelDesc& k, uint32_t ks, SmRes& r) {
  const uint32_t nwm = amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const uint32_t max_cta = amin<uint32_t>(c.max_cta_per_sm, kMaxCta);
  // counted resources: closed form
  uint32_t n = k.cta_per_sm > s.n_cta_k[ks] ? k.cta_per_sm - s.n_cta_k[ks] : 0u;
  n = amin<uint32_t>(n, max_cta > r.ctas ? max_cta - r.ctas : 0u);
  if (k.thr_cta) n = amin<uint32_t>(n, c.max_threads_per_sm > r.thr ? (c.max_threads_per_sm - r.thr) / k.thr_cta : 0u);
  if (k.regs_cta) n = amin<uint32_t>(n, c.regs_per_sm > r.regs ? (c.regs_per_sm - r.regs) / k.regs_cta : 0u);
  if (k.shmem_per_cta) n = amin<uint32_t>(n, k.shmem_cap > r.shmem ? (k.shmem_cap - r.shmem) / k.shmem_per_cta : 0u);
  // warps: first-fit placement of equal CTAs = as many as fit in each free
  // run, lowest run first (one pass over the runs of the free mask)
  const uint32_t wpc = k.warps_per_cta;
  uint32_t placed = 0;
  if (n && wpc && wpc <= nwm) {
    uint64_t freem = ~r.wmask & (nwm >= 64 ? ~0ull : ((1ull << nwm) - 1));
    const uint64_t one = wpc >= 64 ? ~0ull : ((1ull << wpc) - 1);
    while (freem && placed < n) {
      const uint32_t b0 = (uint32_t)ffs64(freem);
      const uint64_t rest = b0 ? (freem >> b0) : freem;
      const uint32_t len = ~rest ? (uint32_t)ffs64(~rest) : 64u - b0;
      uint32_t fit = len / wpc;
      if (fit > n - placed) fit = n - placed;
      for (uint32_t j = 0; j < fit; ++j) r.wmask |= one << (b0 + j * wpc);
      placed += fit;
      freem = (b0 + len >= 64) ? 0ull : (freem & (~0ull << (b0 + len)));
    }
  }
  r.ctas += placed;
  r.thr += placed * k.thr_cta;
  r.regs += placed * k.regs_cta;
  r.shmem += placed * k.shmem_per_cta;
  return placed;
}

// kernel slot (re)initialisation of an SM: first epoch after a launch
template <class P, class S>
SIM_HDI void sm_kernels_init(S& s, const SmCtx& x) {
  const KernelTab& kt = *x.kt;
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k) {
    if (!(kt.active >> k & 1u) || s.k_uid[k] == kt.k[k].uid) continue;
    s.k_uid[k] = kt.k[k].uid;
    s.next_cta[k] = 0;
    for (int xi = 0; xi < kMaxXcd; ++xi) s.next_ctax[k][xi] = 0;
    if (kt.k[k].flush_l1 & 1u) {
      P::each(kMaxL1Lines, [&](int i) {
        s.l1[i].valid = 0;
        s.l1[i].dirty = 0;
      });
      P::sync();
    }
    if (kt.k[k].flush_l1 & 2u) {
      // the dispatch's acquire invalidates the SQC (instruction and scalar
      // data caches): every kernel starts them cold (SQC_ICACHE_MISSES repeat
      // per launch of the same kernel on MI355X)
      P::each(kMaxIL1Lines, [&](int i) { s.il1[i].valid = 0; });
      P::each(kMaxCL1Lines, [&](int i) { s.cl1[i].valid = 0; });
      // fetch-block tags (bit 0 set) go; a warp waiting for a code line
      // (WF_IMISS, bit 0 clear) keeps the line its fill will match
      P::each(kMaxWarps, [&](int w) {
        if (s.w_iline[w] & 1ull) s.w_iline[w] = 0;
      });
      P::sync();
    }
  }
}

// one epoch of one SM: [t0, t1) core cycles
template <class P, class S>
SIM_HDI void sm_epoch(S& s, const SmCtx& x, const EpochPub& pub, uint32_t prev,
                      uint64_t t0, uint64_t t1, const Pkt* inbox, const uint32_t* incnt, uint32_t in_cap,
                      uint32_t n_sub, uint64_t epoch_idx, const uint64_t* rep_dst = nullptr) {
  const SimCfg& c = *x.cfg;
  sm_kernels_init<P>(s, x);
  if (c.link_contention == 2 && x.rt_st) {
    // the injection queue the previous epoch's router pass left (HasBuffer)
    const uint32_t cpc = c.cores_per_cluster ? c.cores_per_cluster : 1;
    s.inj_t0_fs = core_fs(c, t0);
    s.inj_allow0 = rt_inj_allow0(c, x.rt_st, 0, s.id / cpc, fdiv(s.inj_t0_fs, c.dv_icnt));
    s.inj_used = 0;
  }
  // 0. cycles [s.cycle, t0) were fast-forwarded by epoch_decide (nothing could
  //    happen in them): account them exactly like quiet cycles
  if (t0 > s.cycle && (s.n_cta_active || !sm_idle(s))) sm_skip<P>(s, c, t0 - s.cycle, s.cycle);
  s.min_emit = ~0ull;
  // 1. arrivals (replies injected by the memory side last epoch)
  P::prof(12);
  //    (skipped when no channel put a reply for this SM last epoch)
  if (dst_maybe(rep_dst, s.id))
    gather_sorted<P>(inbox, incnt, s.id, n_sub, in_cap, core_fs(c, t0), s.inq, kInQ, s.inq_head, s.inq_n,
                     s_scratch_key(s), s_scratch_ref(s), s_scratch_rank(s), kInQ);
  // 2. CTA dispatch (state published at the previous boundary)
  P::prof(13);
  {
    // rotation by simulated time (t0 / epoch length), not by the epoch counter,
    // so fast-forwarded epochs leave the CTA -> SM assignment unchanged
    const KernelTab& kt = *x.kt;
    uint8_t order[kMaxConc];
    const uint32_t nk = slot_order(kt, order);
    for (uint32_t i = 0; i < nk; ++i)
      if (t0 >= kt.k[order[i]].ready_cycle) {
        const uint32_t rot = (uint32_t)(fdiv(t0, c.dv_epoch) % c.n_sm);
        if (c.n_xcd > 1) cta_dispatch_xcd<P>(s, x, order[i], pub.sm[prev], c.n_sm, rot);
        else cta_dispatch<P>(s, x, order[i], pub.sm[prev], c.n_sm, rot);
      }
  }
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
          P::prof(44);
          const uint64_t nx = P::uni(sm_quiet_until<P>(v, c, *x.kt, t, t1));
          if (nx > t) {
            P::prof(45);
            sm_skip<P>(v, c, nx - t, t);
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
template <class P, class S>
SIM_HDI void sm_publish(S& s, const SmCtx& x, EpochPub& pub, uint32_t cur) {
  const SimCfg& c = *x.cfg;
  // destinations written this epoch (none when no packet was injected: every
  // injection lowers min_emit); this parity's cells are rewritten only if
  // they or the last write to them hold packets (pub_nz bit `cur`)
  uint64_t dm0 = 0, dm1 = 0;
  if (P::uni(s.min_emit) != ~0ull) {
    dm0 = P::vor((int)c.n_subpart, [&](int d) -> uint64_t { return (s.ocnt[d] && !(d & 64)) ? 1ull << (d & 63) : 0; });
    dm1 = P::vor((int)c.n_subpart, [&](int d) -> uint64_t { return (s.ocnt[d] && (d & 64)) ? 1ull << (d & 63) : 0; });
  }
  const uint32_t nzb = 1u << cur, nz = P::uni((uint32_t)s.pub_nz);
  if ((dm0 | dm1) || (nz & nzb)) {
    P::each((int)c.n_subpart, [&](int d) {
      x.outcnt[(uint64_t)d * x.n_src_sm + s.id] = s.ocnt[d];
      s.ocnt[d] = 0;
    });
    P::sync();
  }
  s.pub_nz = (dm0 | dm1) ? (nz | nzb) : (nz & ~nzb);
  // CTA requests per kernel, oldest kernel first: each kernel asks for what
  // is left after the older ones' requests (a request the dispatch does not
  // fill is simply renewed at the next boundary)
  const KernelTab& kt = *x.kt;
  uint8_t order[kMaxConc];
  const uint32_t nk = slot_order(kt, order);
  SmRes r{s.cta_wmask, s.n_cta_active, s.used_thr, s.used_regs, s.used_shmem};
  uint32_t req = 0, kbusy = 0;
  uint64_t reqk = 0;
  bool all_dispatched = true;
  uint32_t other = 0;  // kernels holding (or promised) this SM's resources
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
    if (s.n_cta_k[k]) kbusy |= 1u << k;
  other = kbusy;
  for (uint32_t i = 0; i < nk; ++i) {
    const uint32_t k = order[i];
    const KernelDesc& kd = kt.k[k];
    if (s.next_cta[k] >= kd.n_cta) continue;
    all_dispatched = false;
    // without -gpgpu_concurrent_kernel_sm an SM runs one kernel at a time
    if (!kt.mix && (other & ~(1u << k))) continue;
    const uint32_t n = sm_cta_fit(s, c, kd, k, r);
    if (n) {
      req |= 1u << k;
      reqk |= (uint64_t)n << (8 * k);
      other |= 1u << k;
    }
  }
  const uint32_t idle = (all_dispatched && sm_idle(s)) ? 1u : 0u;
  uint64_t nx = ~0ull;
  if (c.event_skip && (s.n_cta_active || !sm_idle(s)))
    nx = core_fs(c, sm_quiet_until<P>(s, c, kt, s.cycle, s.cycle + kSkipHorizon));
  nx = amin(nx, s.min_emit);
  UnitPub u;
  u.next = nx;
  u.prog = s.last_progress;
  u.insn = s.sget(SK(thread_insn));
  u.req = req;
  u.idle = (uint16_t)idle;
  u.kbusy = (uint8_t)kbusy;
  u.pad8 = 0;
  u.drained = sm_idle(s) ? 1u : 0u;
  u.ctas = (uint32_t)s.sget(SK(ctas_done));
  u.reqk = reqk;
  u.dmask[0] = dm0;
  u.dmask[1] = dm1;
  P::one([&] {
    pub.sm[cur][s.id] = u;
    if (s.id == 0)
      for (int k = 0; k < kMaxConc; ++k) {
        pub.next_cta[cur][k] = s.next_cta[k];
        for (int xi = 0; xi < kMaxXcd; ++xi) pub.next_ctax[cur][k][xi] = s.next_ctax[k][xi];
      }
  });
}

// one epoch of one memory channel
template <class P>
SIM_HDI void chan_epoch(ChanState& ch, const MemCtx& x, const Pkt* inbox, const uint32_t* incnt,
                        uint32_t in_cap, uint64_t t0_fs, const uint64_t* req_dst = nullptr) {
  P::prof(20);
  ch.min_emit = ~0ull;
  if (x.cfg->link_contention == 2 && x.rt_st) {
    const SimCfg& c = *x.cfg;
    ch.inj_t0_fs = t0_fs;
    for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
      ch.sp[j].inj_allow0 = rt_inj_allow0(c, x.rt_st, 1, c.n_clusters + ch.id * c.n_sub_per_mem + j, fdiv(t0_fs, c.dv_icnt));
      ch.sp[j].inj_used = 0;
    }
  }
  mem_gather<P>(ch, *x.cfg, x, inbox, incnt, in_cap, t0_fs, req_dst);
  P::one([&] {
    for (uint32_t j = 0; j < x.cfg->n_sub_per_mem; ++j) ch.sp[j].st.icnt_backlog += ch.sp[j].ovf_n;
  });
  P::prof(24);
  mem_window<P>(ch, x);
  P::prof(25);
}

template <class P>
SIM_HDI void chan_publish(ChanState& ch, const MemCtx& x, EpochPub& pub, uint32_t cur) {
  uint64_t dm[2] = {0, 0};
  mem_publish<P>(ch, *x.cfg, x.outcnt, cur, dm);
  uint32_t idle = chan_idle(ch, *x.cfg) ? 1u : 0u;
  uint64_t nx = ~0ull;
  if (x.cfg->event_skip) nx = chan_next_event(ch, *x.cfg, amin(ch.t_dram, amin(ch.t_l2, ch.t_icnt)));
  nx = amin(nx, ch.min_emit);
  UnitPub u;
  u.next = nx;
  u.prog = 0;
  u.insn = 0;
  u.req = 0;
  u.idle = (uint16_t)idle;
  u.kbusy = 0;
  u.pad8 = 0;
  u.drained = idle;
  u.ctas = 0;
  u.reqk = 0;
  u.dmask[0] = dm[0];
  u.dmask[1] = dm[1];
  P::one([&] { pub.ch[cur][ch.id] = u; });
}

// every participant computes the same decision from the published state
template <class P>
SIM_HDI EpochDecision epoch_decide(const SimCfg& c, const EpochPub& pub, uint32_t cur, uint64_t t1,
                                   const KernelTab& kt, uint64_t epoch_idx, uint64_t max_cycle) {
  EpochDecision d;
  // one pass over every unit's record (one load per unit), then reductions
  uint32_t nbusy = 0, undrained = 0, cbusy = 0, ctas = 0, reqs = 0, kbusy = 0;
  uint64_t sm_next = ~0ull, ch_next = ~0ull, prog = 0, insn = 0;
  uint64_t rq0 = 0, rq1 = 0, rp0 = 0, rp1 = 0;
  P::lane_loop((int)c.n_sm, [&](int j) {
    const UnitPub u = pub.sm[cur][j];
    rq0 |= u.dmask[0];
    rq1 |= u.dmask[1];
    insn += u.insn;
    ctas += u.ctas;
    nbusy += u.idle ? 0u : 1u;
    undrained += u.drained ? 0u : 1u;
    reqs |= u.req;
    kbusy |= u.kbusy;
    sm_next = amin<uint64_t>(sm_next, u.next);
    prog = amax<uint64_t>(prog, u.prog & ((1ull << 56) - 1));  // progress stamps are < 2^56
  });
  P::lane_loop((int)c.n_mem, [&](int j) {
    const UnitPub u = pub.ch[cur][j];
    rp0 |= u.dmask[0];
    rp1 |= u.dmask[1];
    cbusy += u.idle ? 0u : 1u;
    ch_next = amin<uint64_t>(ch_next, u.next);
  });
  nbusy = P::uni(P::red_sum(nbusy));
  undrained = P::uni(P::red_sum(undrained));
  reqs = P::uni(P::red_or(reqs));
  kbusy = P::uni(P::red_or(kbusy));
  cbusy = P::uni(P::red_sum(cbusy));
  sm_next = P::uni(P::red_min64(sm_next));
  ch_next = P::uni(P::red_min64(ch_next));
  prog = P::uni(P::red_max64(prog));
  auto or64 = [&](uint64_t v) -> uint64_t {
    return (uint64_t)P::uni(P::red_or((uint32_t)v)) | (uint64_t)P::uni(P::red_or((uint32_t)(v >> 32))) << 32;
  };
  d.req_dst[0] = or64(rq0);
  d.req_dst[1] = or64(rq1);
  d.rep_dst[0] = or64(rp0);
  d.rep_dst[1] = or64(rp1);
  // per kernel slot: fully dispatched, launch latency, completion
  const uint32_t active = kt.active;
  uint32_t undisp = 0, cut = 0, refill = 0;
  uint64_t ready_min = ~0ull, ready_req = ~0ull, ready_max = 0;
  for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k) {
    if (!(active >> k & 1u)) continue;
    const KernelDesc& kd = kt.k[k];
    ready_max = amax<uint64_t>(ready_max, kd.ready_cycle);
    if (pub.next_cta[cur][k] < kd.n_cta) {
      undisp |= 1u << k;
      if (kd.cta_avail < kd.n_cta && dispatch_bound(c, kd, pub.next_cta[cur][k], pub.next_ctax[cur][k]) >= kd.cta_avail)
        refill = 1;
      ready_min = amin<uint64_t>(ready_min, kd.ready_cycle);
      if (reqs >> k & 1u) ready_req = amin<uint64_t>(ready_req, amax<uint64_t>(t1, kd.ready_cycle));
    } else if (kd.stop_when_issued) {
      cut = 1;
    }
  }
  // a kernel completes when all its CTAs were dispatched and have finished;
  // the last running kernel also waits for the SMs to drain (write-backs,
  // instruction fetches), as the whole GPU going idle ends a serial kernel
  uint32_t done = active & ~undisp & ~kbusy;
  if (done == active && nbusy != 0) done = 0;
  d.done = done;
  d.all_idle = (nbusy == 0 && cbusy == 0) ? 1u : 0u;
  d.next_start = t1;
  d.deadlock = 0;
  // run caps checked while kernels run (reference gpgpu_sim::active,
  // gpu-sim.cc:1071-1094): instructions, completed CTAs, issued CTAs
  d.limit = 0;
  d.refill = refill;
  if (c.max_insn && P::uni(P::red_sum64(insn)) >= c.max_insn) d.limit = 1;
  if (c.max_completed_cta && P::uni(P::red_sum(ctas)) >= c.max_completed_cta) d.limit = 1;
  if (cut) d.limit = 1;
  // fast-forward over the kernel launch latency when nothing is in flight
  if (undisp && cbusy == 0 && t1 < ready_min && undrained == 0) {
    uint64_t E = c.icnt_latency;
    uint64_t skip = fdiv(ready_min - t1, c.dv_epoch) * E;
    d.next_start = t1 + skip;
  }
  // Whole-epoch fast-forward (conservative PDES with exact next-event times):
  // the earliest instant any SM or channel can change state, any packet in
  // flight arrives, or the next CTA can be dispatched bounds how far every
  // participant can jump; epochs wholly before it are skipped.  With no
  // pending event at all (a deadlock) nothing is skipped.
  if (c.event_skip && !d.done) {
    uint64_t ev = amin(sm_next, ch_next);
    if (ready_req != ~0ull) ev = amin(ev, core_fs(c, ready_req));
    if (ev != ~0ull) {
      const uint64_t E = c.icnt_latency;
      const uint64_t tc = core_cyc(c, ev);  // the next epoch may start no later than this
      if (tc >= t1 + E) {
        uint64_t s = t1 + fdiv(tc - t1, c.dv_epoch) * E;
        if (max_cycle && s > max_cycle) s = max_cycle > t1 ? t1 + (max_cycle - t1 + E - 1) / E * E : t1;
        if (s > d.next_start) d.next_start = s;
      }
    }
  }
  if (c.deadlock_window && nbusy && (fdiv(t1, c.dv_epoch) & 63) == 0) {
    // newest progress stamp over all SMs
    const uint64_t last = prog;
    if (t1 > last + c.deadlock_window && t1 > ready_max + c.deadlock_window) d.deadlock = 1;
  }
  (void)epoch_idx;
  return d;
}

}  // namespace asim
