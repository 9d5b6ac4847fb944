// Input-queued router microarchitecture of -network_mode 1 topologies
// (-icnt_link_contention 2): virtual channels, credit flow control, separable
// / iSLIP switch allocation with internal speedup, wormhole switching.
//
// Reference: intersim2/routers/iq_router.cpp (input buffers per VC, route /
// VC-allocation / switch-allocation / traversal pipeline, credits),
// allocators/islip.cpp, separable_input_first.cpp, separable_output_first.cpp,
// buffer_state.cpp (downstream VC ownership and credit counts) and
// gputrafficmanager.cpp (one network per subnet: requests and replies never
// share a router).  The reference steps every router every interconnect cycle
// in lock step with the cores; here the network is simulated cycle by cycle
// once per PDES epoch, over the packets injected in that epoch:
//
//  * every directed link of the topology (icnt_links.h numbering: the output
//    port of the router it leaves) feeds one input unit of the router it
//    enters, with V virtual channels of B flits; every node has an injection
//    input unit; a route's last link ejects into the destination node;
//  * a head flit that reaches an input VC is eligible for the switch after
//    routing + VC allocation + switch allocation delay (hop_icnt - 1), a body
//    flit after the switch-allocation delay; a head needs a free VC on its
//    output's downstream unit (VC and switch allocation are combined: the VC
//    is taken when the head wins the switch), every flit a credit there;
//  * each switch pass matches inputs to outputs with the configured
//    allocator (alloc_iters iterations; iSLIP moves its pointers on first-
//    iteration accepts only); internal speedup S runs S passes per cycle
//    (fractional speedups accumulate), the output buffer drains one flit per
//    cycle onto its link;
//  * a credit returns credit_delay + 1 cycles after its flit leaves the
//    buffer; a downstream VC is released when the tail flit leaves the
//    upstream router (wait_for_tail_credit = 0).
//
// Across epochs the network carries its links' and input units' busy times,
// the sources' injection times and the allocators' pointers (the state
// image); buffers are empty at every epoch start because every packet of an
// epoch is simulated to its arrival (earlier epochs' traffic has priority
// over later epochs').  A packet's extra delay over its uncontended
// traversal -- head latency plus serialisation -- is added to its arrival
// time, so the PDES lookahead (the uncontended minimum) still holds.
//
// The same pass runs open loop over synthetic traffic (driver/icnt_bench.cc,
// Booksim's standalone mode): there every packet is known up front and the
// simulation is exact cycle by cycle.
//
// Sequential and policy-generic (P::one): the CPU and GPU engines produce
// identical results.
#pragma once
#include "icnt_links.h"

namespace asim {

constexpr uint32_t kRtNone = 0xffffffffu;
constexpr uint32_t kRtUnrouted = 0x7fffffffu;  // an adaptive head's next link, not chosen yet
constexpr uint32_t kRtMaxPktBytes = 136;  // 8 B header + 128 B of data
constexpr uint32_t kRtOutSlack = 16;      // output-buffer flits a speedup > 1 may queue ahead of its link
constexpr uint64_t kMaxIcntScratchWords = 1ull << 28;  // 1 GiB of per-epoch router-pass scratch

enum RtAlloc : uint8_t {
  RT_ISLIP = 0,
  RT_SEP_INPUT_FIRST = 1,
  RT_SEP_OUTPUT_FIRST = 2,
  RT_WAVEFRONT = 3,  // diagonals of the request matrix from a priority diagonal that rotates every cycle
  RT_MAX_SIZE = 4,   // maximum matching (augmenting paths)
  RT_PIM = 5,        // parallel iterative matching (random grants / accepts, hashed from the cycle)
  RT_LOA = 6,        // lonely output: the side with the fewest requests wins
};

// deterministic "random" number of parallel iterative matching: the same on
// every host and engine
SIM_HDI uint64_t rt_hash(uint64_t a, uint64_t b) {
  uint64_t z = a * 0x9e3779b97f4a7c15ull ^ (b + 0x632be59bd9b4e019ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// interconnect nodes of the topology
SIM_HDI uint64_t icnt_node_count(const SimCfg& c) {
  const uint32_t k = c.topo_k ? c.topo_k : 2, n = c.topo_n ? c.topo_n : 1;
  const uint64_t kn = ipow(k, n);
  const uint32_t conc = c.topo_conc ? c.topo_conc : 1;
  return (c.topo == TOPO_CMESH || c.topo == TOPO_FLATFLY) ? kn * conc : kn;
}

// the longest route (links) of the topology
SIM_HDI uint32_t icnt_max_route(const SimCfg& c) {
  const uint32_t k = c.topo_k ? c.topo_k : 2, n = c.topo_n ? c.topo_n : 1;
  switch (c.topo) {
    case TOPO_FLY: return n;
    case TOPO_CMESH:
    case TOPO_MESH: return n * (k - 1) + 1;
    case TOPO_TORUS: return n * (k / 2) + 1;
    case TOPO_FATTREE: return 2 * n - 1;
    default: return n + 1;
  }
}

SIM_HDI uint32_t rt_flits(const SimCfg& c, uint32_t bytes) {
  const uint32_t f = (bytes + c.flit_size - 1) / c.flit_size;
  return f ? f : 1;
}

// one subnet's network
struct RtDims {
  uint32_t N, L, U, V, B, H;  // nodes, links, input units (N + L), VCs, flits per VC, longest route
  uint32_t np, nf;            // packet and flit capacity of a pass
};

SIM_HDI RtDims rt_dims(const SimCfg& c, uint32_t max_pkts, uint32_t max_flits_per_pkt) {
  RtDims d;
  d.N = (uint32_t)icnt_node_count(c);
  d.L = (uint32_t)icnt_link_count(c);
  d.U = d.N + d.L;
  d.V = c.rt_vcs ? c.rt_vcs : 1;
  d.B = c.rt_buf ? c.rt_buf : 1;
  d.H = icnt_max_route(c);
  if (c.rt_route == 2) d.H = 2 * d.H;  // Valiant: two dimension-order legs
  d.np = max_pkts;
  d.nf = max_pkts * max_flits_per_pkt;
  return d;
}

// persistent words (u64) of one subnet: link_next[L], gptr[L], in_free[U],
// aptr[U], inj_next[N]
SIM_HDI uint64_t rt_state_words(const RtDims& d) { return 2ull * d.L + 2ull * d.U + d.N; }

// scratch (u32 words) of one pass
struct RtWork {
  uint32_t *src, *dst, *nfl, *fbase, *roff, *nh, *next, *bidx, *pcur;
  uint64_t *tinj, *tarr;
  uint64_t* ready;
  uint32_t *fpk, *fhop;
  uint32_t* route;
  uint64_t* crt;
  uint32_t* crv;
  uint32_t *vhead, *vcnt, *vown, *vout, *vocc;
  uint32_t* ring;
  uint32_t *act, *actf;
  uint32_t *shead, *stail, *sfl, *svc, *slist, *sflag;
  uint32_t *rq_u, *rq_v, *rq_l;
  uint32_t *g_in, *g_key, *g_tag, *a_l, *a_v, *a_key, *a_tag, *m_u, *m_l;
  uint32_t *rq_k, *rq_o, *gb, *ge, *ocnt, *vis, *st_u, *st_e;  // wavefront order, max-size search, LOA counts
  // an explicit network (Booksim anynet, driver/icnt_bench.cc; nullptr: the
  // topology's own routes and the uniform channel latency): the route of
  // node pair (a, b) is rt_links[rt_off[a * N + b] .. rt_off[a * N + b + 1]),
  // link l's channel latency lat[l], node n's injection channel inj_lat[n]
  const uint32_t *rt_off, *rt_links;
  const uint16_t *lat, *inj_lat;
};

// carve the scratch of a pass out of `base` (nullptr: size only); returns
// its u32 words
SIM_HDI uint64_t rt_carve(const RtDims& d, uint32_t* base, RtWork* w) {
  uint64_t off = 0;
  auto take32 = [&](uint64_t n) -> uint32_t* {
    uint32_t* p = base ? base + off : nullptr;
    off += n;
    return p;
  };
  auto take64 = [&](uint64_t n) -> uint64_t* {
    off = (off + 1) & ~1ull;  // 8-byte aligned
    uint64_t* p = base ? reinterpret_cast<uint64_t*>(base + off) : nullptr;
    off += 2 * n;
    return p;
  };
  const uint64_t uv = (uint64_t)d.U * d.V, hops = (uint64_t)d.nf * d.H;
  RtWork t{};
  t.tinj = take64(d.np);
  t.tarr = take64(d.np);
  t.ready = take64(d.nf);
  t.crt = take64(hops);
  t.src = take32(d.np);
  t.dst = take32(d.np);
  t.nfl = take32(d.np);
  t.fbase = take32(d.np);
  t.roff = take32(d.np);
  t.nh = take32(d.np);
  t.next = take32(d.np);
  t.bidx = take32(d.np);
  t.pcur = take32(d.np);
  t.fpk = take32(d.nf);
  t.fhop = take32(d.nf);
  t.route = take32((uint64_t)d.np * d.H);
  t.crv = take32(hops);
  t.vhead = take32(uv);
  t.vcnt = take32(uv);
  t.vown = take32(uv);
  t.vout = take32(uv);
  t.vocc = take32(uv);
  t.ring = take32(uv * d.B);
  t.act = take32(d.U);
  t.actf = take32(d.U);
  t.shead = take32(d.N);
  t.stail = take32(d.N);
  t.sfl = take32(d.N);
  t.svc = take32(d.N);
  t.slist = take32(d.N);
  t.sflag = take32(d.N);
  t.rq_u = take32(uv);
  t.rq_v = take32(uv);
  t.rq_l = take32(uv);
  t.g_in = take32(d.L);
  t.g_key = take32(d.L);
  t.g_tag = take32(d.L);
  t.m_l = take32(d.L);
  t.a_l = take32(d.U);
  t.a_v = take32(d.U);
  t.a_key = take32(d.U);
  t.a_tag = take32(d.U);
  t.m_u = take32(d.U);
  t.rq_k = take32(uv);
  t.rq_o = take32(uv);
  t.gb = take32(d.U);
  t.ge = take32(d.U);
  t.ocnt = take32(d.L);
  t.vis = take32(d.L);
  t.st_u = take32((uint64_t)d.U + 1);
  t.st_e = take32((uint64_t)d.U + 1);
  if (w) *w = t;
  return off + 2;
}

// uncontended traversal of a packet (icnt cycles): head latency of its
// route plus the serialisation of its body flits
SIM_HDI uint64_t rt_uncontended(const SimCfg& c, uint32_t routers, uint32_t nfl) {
  return (uint64_t)routers * c.hop_icnt + (uint64_t)(routers + 1) * c.chan_icnt + (nfl - 1);
}

// Simulate the `np` packets already in w (src, dst, nfl, tinj) through one
// subnet whose persistent state is `st` (rt_state_words); fills w.tarr (the
// tail flit's arrival, icnt cycles) and returns the number of packets that
// could not be delivered (a routing deadlock: they get their uncontended
// traversal after the last delivery).  Single-threaded.
// Router activity of a pass (the inputs of Booksim's power module,
// intersim2/power/power_module.cpp): act[RT_ACT_*] when `act` is given.
enum RtAct : int {
  RT_ACT_BUF_WRITE = 0,  // flits written into an input VC buffer (injection included)
  RT_ACT_BUF_READ,       // flits read out of an input VC buffer = crossbar traversals
  RT_ACT_LINK,           // flits onto a router-to-router link
  RT_ACT_EJECT,          // flits onto an ejection link
  RT_ACT_SA_REQ,         // switch-allocator requests
  RT_ACT_CREDIT,         // credits returned upstream
  RT_ACT_PASSES,         // switch passes run
  RT_ACT_COUNT
};

SIM_HDN uint32_t rt_simulate(const SimCfg& c, const RtDims& d, uint64_t* st, const RtWork& w, uint32_t np,
                             uint64_t* act = nullptr) {
  uint64_t* link_next = st;
  uint64_t* gptr = st + d.L;
  uint64_t* in_free = st + 2 * d.L;
  uint64_t* aptr = st + 2 * d.L + d.U;
  uint64_t* inj_next = st + 2 * d.L + 2 * d.U;
  const uint32_t V = d.V, B = d.B, N = d.N, L = d.L, U = d.U;
  const uint64_t head_delay = c.hop_icnt > 0 ? c.hop_icnt - 1u : 0u, body_delay = c.rt_sa, chan = c.chan_icnt;
  const uint64_t slack = c.rt_speedup_q8 > 256 ? kRtOutSlack : 0;
  const uint32_t iters = c.rt_iters ? c.rt_iters : 1;
  const bool dateline = c.topo == TOPO_TORUS && V >= 2;
  const uint32_t tk = c.topo_k ? c.topo_k : 2, tn = c.topo_n ? c.topo_n : 1;
  // minimal adaptive routing on meshes: VC 0 is the dimension-order escape
  // channel, VCs 1.. are adaptive (Duato); needs >= 2 VCs
  const bool adaptive = c.rt_route == 1 && (c.topo == TOPO_MESH || c.topo == TOPO_CMESH) && V >= 2;
  const uint32_t aconc = c.topo == TOPO_CMESH ? (c.topo_conc ? c.topo_conc : 1) : 1, aP = 2 * tn + aconc;
  // Valiant (mesh): dimension order to a random intermediate router, then
  // dimension order to the destination; the second leg on the upper half of
  // the VCs (two classes keep the two legs' channel dependences acyclic)
  const bool valiant = c.rt_route == 2 && (c.topo == TOPO_MESH || c.topo == TOPO_CMESH) && V >= 2;
  // ---- routes, flits, source queues (injection order: time, then packet) ----
  for (uint32_t s = 0; s < N; ++s) {
    w.shead[s] = w.stail[s] = kRtNone;
    w.sfl[s] = 0;
    w.svc[s] = kRtNone;
    w.sflag[s] = 0;
  }
  uint32_t nf = 0, nsrc = 0;
  for (uint32_t p = 0; p < np; ++p) {
    w.roff[p] = p * d.H;
    uint32_t h = 0, dim = ~0u, crossed = 0;
    if (adaptive) {
      // the head chooses every hop as it goes (adapt_choice): the minimal
      // route's length is known, its links are not
      h = icnt_routers(c, w.src[p], w.dst[p]);
      for (uint32_t i = 0; i < d.H; ++i) w.route[p * d.H + i] = kRtUnrouted;
      w.pcur[p] = w.src[p] / aconc;
    } else if (valiant) {
      // the intermediate router: a hash of the packet's source, destination
      // and injection time (reproducible on every engine)
      const uint32_t nr = (uint32_t)ipow(tk, tn);
      const uint32_t mid = (uint32_t)(rt_hash(w.tinj[p] * 1000003u + w.src[p], w.dst[p]) % nr);
      const uint32_t mid_node = mid * aconc;
      uint32_t leg1 = 0;
      icnt_route(c, w.src[p], mid_node, [&](uint32_t l) {
        leg1 = l;  // (the last link is mid's ejection: dropped below)
        if (h < d.H) w.route[p * d.H + h] = l;
        ++h;
      });
      (void)leg1;
      --h;  // drop the ejection link into the intermediate node
      icnt_route(c, mid_node, w.dst[p], [&](uint32_t l) {
        if (h < d.H) w.route[p * d.H + h] = l | 1u << 31;
        ++h;
      });
    } else if (w.rt_off) {
      const uint64_t pr = (uint64_t)w.src[p] * N + w.dst[p];
      for (uint32_t i = w.rt_off[pr]; i < w.rt_off[pr + 1]; ++i) {
        if (h < d.H) w.route[p * d.H + h] = w.rt_links[i];
        ++h;
      }
    } else icnt_route(c, w.src[p], w.dst[p], [&](uint32_t l) {
      // torus with >= 2 VCs: dateline classes (the upper half of the VCs
      // after the wrap-around link of the current dimension; reference
      // routefunc.cpp dim_order_torus), kept in the link's top bit
      uint32_t cls = 0;
      if (dateline) {
        const uint32_t P = 2 * tn + 1, port = l % P, cur = l / P;
        if (port < 2 * tn) {
          const uint32_t dd = port / 2;
          if (dd != dim) {
            dim = dd;
            crossed = 0;
          }
          const uint32_t x = (uint32_t)((cur / ipow(tk, dd)) % tk);
          if ((port % 2 == 0 && x == tk - 1) || (port % 2 == 1 && x == 0)) crossed = 1;
          cls = crossed;
        }
      }
      if (h < d.H) w.route[p * d.H + h] = l | cls << 31;
      ++h;
    });
    w.nh[p] = h < d.H ? h : d.H;
    w.fbase[p] = nf;
    for (uint32_t i = 0; i < w.nfl[p]; ++i) {
      w.fpk[nf + i] = p;
      w.fhop[nf + i] = 0;
    }
    nf += w.nfl[p];
    w.tarr[p] = 0;
    const uint32_t s = w.src[p];
    w.next[p] = kRtNone;
    if (w.shead[s] == kRtNone) {
      w.shead[s] = w.stail[s] = p;
      w.sflag[s] = 1;
      w.slist[nsrc++] = s;
    } else if (w.tinj[w.stail[s]] <= w.tinj[p]) {
      w.next[w.stail[s]] = p;
      w.stail[s] = p;
    } else if (w.tinj[p] < w.tinj[w.shead[s]]) {
      w.next[p] = w.shead[s];
      w.shead[s] = p;
    } else {
      uint32_t q = w.shead[s];
      while (w.next[q] != kRtNone && w.tinj[w.next[q]] <= w.tinj[p]) q = w.next[q];
      w.next[p] = w.next[q];
      w.next[q] = p;
    }
  }
  for (uint64_t i = 0; i < (uint64_t)U * V; ++i) {
    w.vhead[i] = w.vcnt[i] = w.vocc[i] = 0;
    w.vown[i] = w.vout[i] = kRtNone;
  }
  for (uint32_t u = 0; u < U; ++u) {
    w.actf[u] = 0;
    w.a_tag[u] = w.m_u[u] = 0;
  }
  for (uint32_t l = 0; l < L; ++l) w.g_tag[l] = w.m_l[l] = w.vis[l] = 0;
  uint32_t dfs = 0;
  uint32_t nact = 0, tag = 0, rtag = 0, cr_r = 0, cr_w = 0, remaining = np, acc = 0;
  auto activate = [&](uint32_t u) {
    if (!w.actf[u]) {
      w.actf[u] = 1;
      w.act[nact++] = u;
    }
  };
  auto push = [&](uint32_t uv, uint32_t f) {
    w.ring[(uint64_t)uv * B + (w.vhead[uv] + w.vcnt[uv]) % B] = f;
    ++w.vcnt[uv];
  };
  // a free VC with room on downstream unit du (kRtNone if none)
  // VC class: dateline (torus) 0 lower / 1 upper half; adaptive 0 escape VC
  // / 1 adaptive VCs; 2 any
  auto free_vc = [&](uint32_t du, uint32_t cls) -> uint32_t {
    uint32_t v0 = 0, v1 = V;
    if (cls < 2 && (dateline || valiant)) {
      v0 = cls ? V / 2 : 0;
      v1 = cls ? V : V / 2;
    } else if (cls < 2 && adaptive) {
      v0 = cls ? 1 : 0;
      v1 = cls ? V : 1;
    }
    for (uint32_t v = v0; v < v1; ++v) {
      const uint32_t i = du * V + v;
      if (w.vown[i] == kRtNone && w.vocc[i] < B) return v;
    }
    return kRtNone;
  };
  // the head of packet p chooses its next link: the productive direction
  // whose downstream unit has an adaptive VC with the most free slots
  // (lowest dimension on ties), else the dimension-order link if its escape
  // VC is free; kRtUnrouted if blocked.  Returns link | class << 31.
  auto adapt_choice = [&](uint32_t p) -> uint32_t {
    const uint32_t cur = w.pcur[p], dst = w.dst[p] / aconc;
    if (cur == dst) return cur * aP + 2 * tn + w.dst[p] % aconc;  // ejection
    uint32_t best = kRtUnrouted, best_free = 0, esc = kRtUnrouted;
    uint64_t pw = 1;
    for (uint32_t dd = 0; dd < tn; ++dd, pw *= tk) {
      const uint32_t x = (uint32_t)((cur / pw) % tk), y = (uint32_t)((dst / pw) % tk);
      if (x == y) continue;
      const uint32_t l = cur * aP + 2 * dd + (y > x ? 0u : 1u), du = N + l;
      if (esc == kRtUnrouted) esc = l;
      for (uint32_t v = 1; v < V; ++v) {
        const uint32_t i = du * V + v;
        if (w.vown[i] == kRtNone && w.vocc[i] < B && B - w.vocc[i] > best_free) {
          best_free = B - w.vocc[i];
          best = l;
        }
      }
    }
    if (best != kRtUnrouted) return best | 1u << 31;
    if (esc != kRtUnrouted && free_vc(N + esc, 0) != kRtNone) return esc;
    return kRtUnrouted;
  };
  uint64_t now = ~0ull;
  for (uint32_t i = 0; i < nsrc; ++i) {
    const uint32_t s = w.slist[i];
    const uint64_t t = w.tinj[w.shead[s]] > inj_next[s] ? w.tinj[w.shead[s]] : inj_next[s];
    if (t < now) now = t;
  }
  while (remaining > 0) {
    bool progress = false;
    // ---- credits that reach their upstream this cycle ----
    while (cr_r < cr_w && w.crt[cr_r] <= now) {
      --w.vocc[w.crv[cr_r]];
      if (act) ++act[RT_ACT_CREDIT];
      ++cr_r;
      progress = true;
    }
    // ---- injection: one flit per source per cycle ----
    {
      uint32_t keep = 0;
      for (uint32_t i = 0; i < nsrc; ++i) {
        const uint32_t s = w.slist[i];
        const uint32_t p = w.shead[s];
        if (p == kRtNone) {
          w.sflag[s] = 0;
          continue;
        }
        w.slist[keep++] = s;
        if (now < w.tinj[p] || now < inj_next[s]) continue;
        if (w.svc[s] == kRtNone) {
          const uint32_t v = free_vc(s, 2);
          if (v == kRtNone) continue;
          w.svc[s] = v;
          w.vown[s * V + v] = p;
        }
        const uint32_t uv = s * V + w.svc[s];
        if (w.vocc[uv] >= B) continue;
        const uint32_t i_f = w.sfl[s], f = w.fbase[p] + i_f;
        push(uv, f);
        if (act) ++act[RT_ACT_BUF_WRITE];
        ++w.vocc[uv];
        w.fhop[f] = 0;
        w.ready[f] = now + (w.inj_lat ? w.inj_lat[s] : chan) + (i_f == 0 ? head_delay : body_delay);
        activate(s);
        inj_next[s] = now + 1;
        progress = true;
        if (++w.sfl[s] == w.nfl[p]) {
          w.vown[uv] = kRtNone;
          w.sfl[s] = 0;
          w.svc[s] = kRtNone;
          w.shead[s] = w.next[p];
        }
      }
      nsrc = keep;
    }
    // ---- switch passes (internal speedup) ----
    acc += c.rt_speedup_q8 ? c.rt_speedup_q8 : 256u;
    const uint32_t passes = acc >> 8;
    acc &= 255u;
    for (uint32_t pass = 0; pass < passes; ++pass) {
      ++rtag;
      // requests: per input unit, per output the VC with the oldest eligible head flit
      uint32_t nrq = 0;
      for (uint32_t i = 0; i < nact; ++i) {
        const uint32_t u = w.act[i];
        if (now < in_free[u]) continue;  // an earlier epoch's flits still leaving (FIFO)
        const uint32_t first = nrq;
        for (uint32_t v = 0; v < V; ++v) {
          const uint32_t uv = u * V + v;
          if (!w.vcnt[uv]) continue;
          const uint32_t f = w.ring[(uint64_t)uv * B + w.vhead[uv]];
          if (w.ready[f] > now) continue;
          const uint32_t p = w.fpk[f], h = w.fhop[f];
          if (adaptive && f == w.fbase[p]) {
            const uint32_t ch = adapt_choice(p);
            if (ch == kRtUnrouted) continue;
            w.route[w.roff[p] + h] = ch;
          }
          const uint32_t rl = w.route[w.roff[p] + h], l = rl & 0x7fffffffu;
          const bool last = h + 1 >= w.nh[p];
          if (!last) {
            const uint32_t du = N + l;
            if (f == w.fbase[p]) {
              if (free_vc(du, rl >> 31) == kRtNone) continue;
            } else if (w.vocc[du * V + w.vout[uv]] >= B) {
              continue;
            }
          }
          const uint64_t dep = link_next[l] > now + 1 ? link_next[l] : now + 1;
          if (dep > now + 1 + slack) continue;
          uint32_t j = first;
          while (j < nrq && w.rq_l[j] != l) ++j;
          if (j == nrq) {
            w.rq_u[nrq] = u;
            w.rq_v[nrq] = v;
            w.rq_l[nrq] = l;
            ++nrq;
          } else {
            const uint32_t g = w.ring[(uint64_t)(u * V + w.rq_v[j]) * B + w.vhead[u * V + w.rq_v[j]]];
            if (w.ready[f] < w.ready[g]) w.rq_v[j] = v;
          }
        }
      }
      if (act) {
        ++act[RT_ACT_PASSES];
        act[RT_ACT_SA_REQ] += nrq;
      }
      if (!nrq) continue;
      // matching
      for (uint32_t it = 0; it < iters; ++it) {
        ++tag;
        bool any = false;
        if (c.rt_alloc == RT_WAVEFRONT || c.rt_alloc == RT_MAX_SIZE) {
          // one-shot allocators: a single iteration finds the whole matching
          if (it > 0) break;
          if (c.rt_alloc == RT_WAVEFRONT) {
            // diagonal (u + l) mod n of the request matrix, from the priority
            // diagonal of this cycle; within a diagonal no two cells share a
            // row or a column
            const uint32_t n = U > L ? U : L, pd = (uint32_t)(now % n);
            for (uint32_t j = 0; j < nrq; ++j) {
              w.rq_k[j] = (w.rq_u[j] + w.rq_l[j] + n - pd) % n;
              uint32_t q = j;  // insertion into the order by (diagonal, request)
              while (q > 0 && w.rq_k[w.rq_o[q - 1]] > w.rq_k[j]) {
                w.rq_o[q] = w.rq_o[q - 1];
                --q;
              }
              w.rq_o[q] = j;
            }
            for (uint32_t q = 0; q < nrq; ++q) {
              const uint32_t j = w.rq_o[q], u = w.rq_u[j], l = w.rq_l[j];
              if (w.a_tag[u] == tag || w.g_tag[l] == tag) continue;
              w.a_tag[u] = w.g_tag[l] = tag;
              w.a_l[u] = l;
              w.a_v[u] = w.rq_v[j];
              w.g_in[l] = u;
            }
          } else {
            // maximum matching: an augmenting path from every input in turn
            // (its requests are contiguous in the request list)
            for (uint32_t j = 0; j < nrq; ++j) {
              if (j == 0 || w.rq_u[j - 1] != w.rq_u[j]) w.gb[w.rq_u[j]] = j;
              w.ge[w.rq_u[j]] = j + 1;
            }
            for (uint32_t j = 0; j < nrq; j = w.ge[w.rq_u[j]]) {
              ++dfs;
              uint32_t sp = 1;
              w.st_u[0] = w.rq_u[j];
              w.st_e[0] = w.gb[w.rq_u[j]];
              while (sp > 0) {
                const uint32_t u = w.st_u[sp - 1], e = w.st_e[sp - 1];
                if (e >= w.ge[u]) {
                  --sp;
                  continue;
                }
                w.st_e[sp - 1] = e + 1;
                const uint32_t l = w.rq_l[e];
                if (w.vis[l] == dfs) continue;
                w.vis[l] = dfs;
                if (w.g_tag[l] != tag) {
                  // free output: flip the path (every frame takes the edge it tried last)
                  for (uint32_t k = sp; k-- > 0;) {
                    const uint32_t uu = w.st_u[k], ee = w.st_e[k] - 1, ll = w.rq_l[ee];
                    w.g_tag[ll] = tag;
                    w.g_in[ll] = uu;
                    w.a_tag[uu] = tag;
                    w.a_l[uu] = ll;
                    w.a_v[uu] = w.rq_v[ee];
                  }
                  break;
                }
                if (sp <= U) {  // the output's input looks for another output
                  w.st_u[sp] = w.g_in[l];
                  w.st_e[sp] = w.gb[w.g_in[l]];
                  ++sp;
                }
              }
            }
          }
        } else if (c.rt_alloc == RT_PIM || c.rt_alloc == RT_LOA) {
          // requests per output (LOA's loneliness) and per input
          for (uint32_t j = 0; j < nrq; ++j) w.ocnt[w.rq_l[j]] = 0;
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.m_u[u] == rtag || w.m_l[l] == rtag) continue;
            ++w.ocnt[l];
            if (j == 0 || w.rq_u[j - 1] != u) w.gb[u] = j;
            w.ge[u] = j + 1;
          }
          const uint64_t seed = now * 0x100000001b3ull + (uint64_t)rtag * 131u + it;
          // outputs grant: PIM uniformly at random (reservoir over the
          // requesters), LOA to the input with the fewest requests
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.m_u[u] == rtag || w.m_l[l] == rtag) continue;
            if (c.rt_alloc == RT_PIM) {
              const uint32_t n = w.g_tag[l] == tag ? w.g_key[l] + 1 : 1;
              if (n == 1 || rt_hash(seed, (uint64_t)l << 20 | n) % n == 0) w.g_in[l] = u;
              w.g_tag[l] = tag;
              w.g_key[l] = n;
            } else {
              const uint32_t key = (w.ge[u] - w.gb[u]) << 20 | (uint32_t)((u + U - gptr[l] % U) % U);
              if (w.g_tag[l] != tag || key < w.g_key[l]) {
                w.g_tag[l] = tag;
                w.g_key[l] = key;
                w.g_in[l] = u;
              }
            }
          }
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.g_tag[l] != tag || w.g_in[l] != u) continue;
            if (c.rt_alloc == RT_PIM) {
              const uint32_t n = w.a_tag[u] == tag ? w.a_key[u] + 1 : 1;
              if (n == 1 || rt_hash(seed + 7, (uint64_t)u << 20 | n) % n == 0) {
                w.a_l[u] = l;
                w.a_v[u] = w.rq_v[j];
              }
              w.a_tag[u] = tag;
              w.a_key[u] = n;
            } else {
              const uint32_t key = w.ocnt[l] << 20 | (uint32_t)((l + L - aptr[u] % L) % L);
              if (w.a_tag[u] != tag || key < w.a_key[u]) {
                w.a_tag[u] = tag;
                w.a_key[u] = key;
                w.a_l[u] = l;
                w.a_v[u] = w.rq_v[j];
              }
            }
          }
        } else if (c.rt_alloc == RT_SEP_INPUT_FIRST) {
          // inputs choose first (accept pointer), then outputs (grant pointer)
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.m_u[u] == rtag || w.m_l[l] == rtag) continue;
            const uint32_t key = (uint32_t)((l + L - aptr[u] % L) % L);
            if (w.a_tag[u] != tag || key < w.a_key[u]) {
              w.a_tag[u] = tag;
              w.a_key[u] = key;
              w.a_l[u] = l;
              w.a_v[u] = w.rq_v[j];
            }
          }
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.a_tag[u] != tag || w.a_l[u] != l || w.m_l[l] == rtag) continue;
            const uint32_t key = (uint32_t)((u + U - gptr[l] % U) % U);
            if (w.g_tag[l] != tag || key < w.g_key[l]) {
              w.g_tag[l] = tag;
              w.g_key[l] = key;
              w.g_in[l] = u;
            }
          }
        } else {
          // outputs grant (grant pointer), inputs accept (accept pointer)
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.m_u[u] == rtag || w.m_l[l] == rtag) continue;
            const uint32_t key = (uint32_t)((u + U - gptr[l] % U) % U);
            if (w.g_tag[l] != tag || key < w.g_key[l]) {
              w.g_tag[l] = tag;
              w.g_key[l] = key;
              w.g_in[l] = u;
            }
          }
          for (uint32_t j = 0; j < nrq; ++j) {
            const uint32_t u = w.rq_u[j], l = w.rq_l[j];
            if (w.g_tag[l] != tag || w.g_in[l] != u) continue;
            const uint32_t key = (uint32_t)((l + L - aptr[u] % L) % L);
            if (w.a_tag[u] != tag || key < w.a_key[u]) {
              w.a_tag[u] = tag;
              w.a_key[u] = key;
              w.a_l[u] = l;
              w.a_v[u] = w.rq_v[j];
            }
          }
        }
        // commit the pairs both sides chose, in request order
        for (uint32_t j = 0; j < nrq; ++j) {
          const uint32_t u = w.rq_u[j], l = w.rq_l[j];
          if (w.a_tag[u] != tag || w.a_l[u] != l || w.g_tag[l] != tag || w.g_in[l] != u) continue;
          if (w.m_u[u] == rtag || w.m_l[l] == rtag) continue;
          w.m_u[u] = rtag;
          w.m_l[l] = rtag;
          any = true;
          progress = true;
          // iSLIP moves its pointers on first-iteration matches only
          if (c.rt_alloc != RT_ISLIP || it == 0) {
            gptr[l] = (u + 1) % U;
            aptr[u] = (l + 1) % L;
          }
          // switch traversal of the head flit of VC (u, a_v[u])
          const uint32_t uv = u * V + w.a_v[u];
          const uint32_t f = w.ring[(uint64_t)uv * B + w.vhead[uv]];
          w.vhead[uv] = (w.vhead[uv] + 1) % B;
          --w.vcnt[uv];
          w.crt[cr_w] = now + 1 + c.rt_credit;
          w.crv[cr_w] = uv;
          ++cr_w;
          in_free[u] = now;
          const uint32_t p = w.fpk[f], h = w.fhop[f], fi = f - w.fbase[p];
          const bool head = fi == 0, tail = fi + 1 == w.nfl[p];
          const uint64_t dep = link_next[l] > now + 1 ? link_next[l] : now + 1;
          link_next[l] = dep + 1;
          if (act) {
            ++act[RT_ACT_BUF_READ];
            ++act[h + 1 < w.nh[p] ? RT_ACT_LINK : RT_ACT_EJECT];
          }
          const uint64_t arr = dep + (w.lat ? w.lat[l] : chan);
          if (h + 1 < w.nh[p]) {
            const uint32_t du = N + l;
            if (head) {
              const uint32_t dv = free_vc(du, w.route[w.roff[p] + h] >> 31);
              w.vout[uv] = dv;
              w.vown[du * V + dv] = p;
            }
            if (adaptive && head) {
              // the head moves one router along dimension port / 2
              const uint32_t port = l % aP, dd = port / 2;
              const uint32_t pw = (uint32_t)ipow(tk, dd);
              w.pcur[p] = port % 2 == 0 ? w.pcur[p] + pw : w.pcur[p] - pw;
            }
            const uint32_t duv = du * V + w.vout[uv];
            ++w.vocc[duv];
            push(duv, f);
            if (act) ++act[RT_ACT_BUF_WRITE];
            w.fhop[f] = h + 1;
            w.ready[f] = arr + (head ? head_delay : body_delay);
            activate(du);
            if (tail) {
              w.vown[duv] = kRtNone;
              w.vout[uv] = kRtNone;
            }
          } else if (tail) {
            w.tarr[p] = arr;
            --remaining;
          }
        }
        if (!any) break;
      }
    }
    // ---- retire empty input units ----
    {
      uint32_t keep = 0;
      for (uint32_t i = 0; i < nact; ++i) {
        const uint32_t u = w.act[i];
        uint32_t cnt = 0;
        for (uint32_t v = 0; v < V; ++v) cnt += w.vcnt[u * V + v];
        if (cnt) {
          w.act[keep++] = u;
        } else {
          w.actf[u] = 0;
        }
      }
      nact = keep;
    }
    if (!remaining) break;
    // ---- next cycle, or the next time anything can move ----
    uint64_t nxt = ~0ull;
    if (progress) {
      nxt = now + 1;
    } else {
      if (cr_r < cr_w) nxt = w.crt[cr_r];
      for (uint32_t i = 0; i < nsrc; ++i) {
        const uint32_t s = w.slist[i], p = w.shead[s];
        if (p == kRtNone) continue;
        const uint64_t t = w.tinj[p] > inj_next[s] ? w.tinj[p] : inj_next[s];
        if (t > now && t < nxt) nxt = t;  // (t <= now: waiting for a credit)
      }
      for (uint32_t i = 0; i < nact; ++i) {
        const uint32_t u = w.act[i];
        for (uint32_t v = 0; v < V; ++v) {
          const uint32_t uv = u * V + v;
          if (!w.vcnt[uv]) continue;
          const uint32_t f = w.ring[(uint64_t)uv * B + w.vhead[uv]];
          uint64_t t = w.ready[f] > in_free[u] ? w.ready[f] : in_free[u];
          const uint32_t l = w.route[w.roff[w.fpk[f]] + w.fhop[f]] & 0x7fffffffu;
          if (l < L && link_next[l] > 1 + slack && link_next[l] - 1 - slack > t) t = link_next[l] - 1 - slack;
          if (t > now && t < nxt) nxt = t;  // (t <= now: waiting for a VC or a credit)
        }
      }
    }
    if (nxt == ~0ull) break;  // nothing can ever move: deadlock
    now = nxt;
  }
  if (remaining) {
    // deadlocked packets: their uncontended traversal after the last event
    for (uint32_t p = 0; p < np; ++p)
      if (!w.tarr[p]) w.tarr[p] = (now > w.tinj[p] ? now : w.tinj[p]) + rt_uncontended(c, w.nh[p], w.nfl[p]);
  }
  return remaining;
}

// ---- injection back-pressure (-icnt_link_contention 2) ----
// The reference refuses a packet whose flits do not fit the node's injection
// queue (InterconnectInterface::HasBuffer, interconnect_interface.cpp:260-272:
// queued flits + the packet's <= input_buffer_size) and the SM's LD/ST unit
// or the L2's reply queue stalls (shader.cc:4554, gpu-sim.cc:1887).  Here the
// network is simulated after each epoch, so an injector sees the queue the
// previous pass left: the source's injection channel takes one flit per
// cycle, so inj_next[node] - t0 flits of earlier traffic are still queued at
// the epoch start t0 (icnt cycles), draining one per cycle.  A packet of
// `nfl` flits may enter at icnt cycle t0 + k while
//   injected_this_epoch + nfl <= rt_inj_allow0 + k,
// rt_inj_allow0 = input_buffer_size - backlog (negative: the queue overflowed).
// Nodes that several SMs share (a cluster) split it: each SM counts its
// flits times the cluster's SMs.
SIM_HDI int64_t rt_inj_allow0(const SimCfg& c, const uint64_t* st, uint32_t subnet, uint32_t node, uint64_t t0_icnt) {
  const RtDims d = rt_dims(c, 0, 0);
  const uint64_t* inj_next = st + (uint64_t)subnet * rt_state_words(d) + 2ull * d.L + 2ull * d.U;
  const uint64_t q = inj_next[node];
  const uint64_t backlog = q > t0_icnt ? q - t0_icnt : 0;
  return (int64_t)c.rt_inbuf - (int64_t)(backlog < (1ull << 40) ? backlog : (1ull << 40));
}

// Scratch words of the epoch pass: both subnets run one after the other
// over the same scratch; a subnet's packets are at most its mailbox cells x
// capacity (icnt_contend's bound).
SIM_HDI RtDims rt_epoch_dims(const SimCfg& c, uint32_t cap_req, uint32_t cap_rep) {
  const uint32_t cap = cap_req > cap_rep ? cap_req : cap_rep;
  return rt_dims(c, c.n_sm * c.n_subpart * cap, rt_flits(c, kRtMaxPktBytes));
}

// The epoch-boundary pass of -icnt_link_contention 2 over this epoch's
// outboxes (same layout and packet order as icnt_contend): `st` holds both
// subnets' persistent state then the two statistics words; `scratch` holds
// rt_carve(rt_epoch_dims) words.
SIM_HDN void rt_epoch_run(const SimCfg& c, Pkt* box_req, const uint32_t* cnt_req, uint32_t cap_req, Pkt* box_rep,
                         const uint32_t* cnt_rep, uint32_t cap_rep, uint64_t* st, uint32_t* scratch) {
  const RtDims d = rt_epoch_dims(c, cap_req, cap_rep);
  RtWork w;
  rt_carve(d, scratch, &w);
  uint64_t* stat = st + 2 * rt_state_words(d);
  const uint32_t ncell = c.n_sm * c.n_subpart;
  const uint32_t cpc = c.cores_per_cluster ? c.cores_per_cluster : 1;
  for (int dir = 0; dir < 2; ++dir) {
    const uint32_t* cnt = dir == 0 ? cnt_req : cnt_rep;
    Pkt* box = dir == 0 ? box_req : box_rep;
    const uint32_t cap = dir == 0 ? cap_req : cap_rep;
    // the packets in cell order (their box slots in w.bidx)
    uint32_t np = 0;
    for (uint32_t cell = 0; cell < ncell; ++cell) {
      for (uint32_t j = 0; j < cnt[cell]; ++j) {
        const Pkt& p = box[(uint64_t)cell * cap + j];
        uint32_t a, b, sm, sub;
        if (dir == 0) {  // request: SM (cell % n_sm) -> sub-partition (cell / n_sm)
          sm = cell % c.n_sm;
          sub = cell / c.n_sm;
          a = sm / cpc;
          b = c.n_clusters + sub;
        } else {  // reply: sub-partition (cell % n_subpart) -> SM (cell / n_subpart)
          sub = cell % c.n_subpart;
          sm = cell / c.n_subpart;
          a = c.n_clusters + sub;
          b = sm / cpc;
        }
        const uint64_t lat = icnt_pkt_lat_fs(c, sm, sub);
        const uint64_t t0 = p.t > lat ? p.t - lat : 0;
        w.src[np] = a;
        w.dst[np] = b;
        const uint32_t nfl = rt_flits(c, p.size ? p.size : 1), nfl_max = rt_flits(c, kRtMaxPktBytes);
        w.nfl[np] = nfl < nfl_max ? nfl : nfl_max;  // the scratch holds nfl_max flits per packet
        w.tinj[np] = fdiv(t0, c.dv_icnt);
        w.bidx[np] = cell * cap + j;
        ++np;
      }
    }
    if (!np) continue;
    const uint32_t lost = rt_simulate(c, d, st + (uint64_t)dir * rt_state_words(d), w, np);
    uint64_t delayed = 0, wait = 0;
    for (uint32_t i = 0; i < np; ++i) {
      const uint64_t base = w.tinj[i] + rt_uncontended(c, icnt_routers(c, w.src[i], w.dst[i]), w.nfl[i]);
      const uint64_t D = w.tarr[i] > base ? w.tarr[i] - base : 0;
      if (D) {
        ++delayed;
        wait += D;
        box[w.bidx[i]].t += D * c.per_icnt;
      }
    }
    stat[0] += delayed;
    stat[1] += wait;
    stat[2] += lost;  // routing deadlock: those packets kept their uncontended latency
  }
}

template <class P>
SIM_HDI void icnt_route_pass(const SimCfg& c, Pkt* box_req, const uint32_t* cnt_req, uint32_t cap_req, Pkt* box_rep,
                             const uint32_t* cnt_rep, uint32_t cap_rep, uint64_t* st, uint32_t* scratch) {
  P::one([&] { rt_epoch_run(c, box_req, cnt_req, cap_req, box_rep, cnt_rep, cap_rep, st, scratch); });
  P::sync();
}

// ---- the engines' entry points: either link model behind one state array ----

// persistent u64 words (statistics words excluded) and u32 scratch words
SIM_HDI uint64_t icnt_state_words(const SimCfg& c, uint32_t cap_req, uint32_t cap_rep) {
  if (c.link_contention == 2) return 2 * rt_state_words(rt_epoch_dims(c, cap_req, cap_rep));
  return icnt_link_count(c);
}
SIM_HDI uint64_t icnt_scratch_words(const SimCfg& c, uint32_t cap_req, uint32_t cap_rep) {
  if (c.link_contention == 2) return rt_carve(rt_epoch_dims(c, cap_req, cap_rep), nullptr, nullptr);
  return (uint64_t)c.n_sm * c.n_subpart * (cap_req > cap_rep ? cap_req : cap_rep);
}

// `st`: icnt_state_words then kIcntStatWords statistics words {delayed
// packets, delay in interconnect cycles, packets of a routing deadlock}
template <class P>
SIM_HDI void icnt_epoch_pass(const SimCfg& c, Pkt* box_req, const uint32_t* cnt_req, uint32_t cap_req, Pkt* box_rep,
                             const uint32_t* cnt_rep, uint32_t cap_rep, uint64_t* st, uint32_t* scratch) {
  if (c.link_contention == 2) {
    icnt_route_pass<P>(c, box_req, cnt_req, cap_req, box_rep, cnt_rep, cap_rep, st, scratch);
  } else {
    icnt_contend<P>(c, box_req, cnt_req, cap_req, box_rep, cnt_rep, cap_rep, st, scratch,
                    st + icnt_link_count(c));
  }
}

}  // namespace asim
