// Link-level contention inside multi-hop interconnect topologies
// (-network_mode 1 with -icnt_link_contention 1).
//
// The reference's intersim2 simulates every router of a Booksim network
// cycle by cycle (intersim2/routers/iq_router.cpp, networks/kncube.cpp,
// fly.cpp, fattree.cpp, flatfly_onchip.cpp): packets that share a link wait
// for it.  The epoch engine prices a packet's route at injection (config.h
// icnt_pkt_lat_fs); this pass adds what the shared links cost.  At every
// epoch boundary the packets injected during the epoch (both directions) are
// walked in a fixed order -- requests then replies, by destination, source
// and injection order -- and each reserves, hop by hop, the directed links of
// its deterministic route (dimension order on meshes / tori, destination-tag
// on butterflies, d-mod-k on fat trees, one hop per differing dimension on
// flattened butterflies) for its flits: a link busy with an earlier
// reservation delays the packet and every later hop.  The last link of every
// route is the destination's ejection link, so arrivals at one destination
// stay in reservation order (its input queue stays time sorted).
//
// Contention only delays packets, so the PDES lookahead (the uncontended
// minimum latency) still holds.  A single-stage butterfly (the crossbar every
// tested config uses) has no internal links: its contention is the ports',
// which the engines model at the endpoints already (the router model of
// -icnt_link_contention 2, icnt_router.h, arbitrates its output ports too).
//
// The pass is policy-generic (P = SeqPar on the CPU engine, WavePar on one
// GPU block) and its order is fixed, so both engines give identical results.
#pragma once
#if !defined(__HIP_DEVICE_COMPILE__)
#include <stdexcept>
#endif
#include "config.h"

namespace asim {

// statistics words behind a link model's persistent state: packets delayed,
// their delay (interconnect cycles), and (router model) packets lost to a
// routing deadlock, which then kept their uncontended latency
constexpr int kIcntStatWords = 3;


constexpr int kMaxPathLinks = 256;
constexpr uint64_t kMaxIcntLinks = 1ull << 22;

SIM_HDI uint64_t ipow(uint32_t k, uint32_t n) {
  uint64_t r = 1;
  for (uint32_t i = 0; i < n; ++i) r *= k;
  return r;
}

// directed links of the topology that the route model names (0: none)
SIM_HDI uint64_t icnt_link_count(const SimCfg& c) {
  if (c.icnt_mode != 1) return 0;
  const uint32_t k = c.topo_k ? c.topo_k : 2, n = c.topo_n ? c.topo_n : 1;
  const uint64_t kn = ipow(k, n);
  switch (c.topo) {
    // stage x router x port; a single-stage fly (a crossbar) has only its
    // output ports, which the router model (icnt_router.h) arbitrates
    case TOPO_FLY: return n <= 1 && c.link_contention != 2 ? 0 : (uint64_t)n * kn;
    case TOPO_CMESH:
    case TOPO_MESH:
    case TOPO_TORUS: return kn * (2ull * n + (c.topo == TOPO_CMESH ? (c.topo_conc ? c.topo_conc : 1) : 1));
    case TOPO_FATTREE: return 2ull * n * kn + kn;  // up, down, ejection
    default:  // flattened butterfly: per dimension and target, + one ejection link per terminal
      return kn * ((uint64_t)n * k + (c.topo_conc ? c.topo_conc : 1));
  }
}

SIM_HDI bool icnt_contention_fits(const SimCfg& c, uint32_t cap_req, uint32_t cap_rep) {
  return (uint64_t)c.n_sm * c.n_subpart <= 65536u && cap_req < 65536u && cap_rep < 65536u;
}
SIM_HDI bool icnt_contention_on(const SimCfg& c) {
  const uint64_t n = icnt_link_count(c);
  return c.link_contention && n > 0 && n <= kMaxIcntLinks;
}

// visit the links of the route from interconnect node a to node b in
// traversal order (the last one ejects into b): emit(link); returns their
// number (== icnt_routers(c, a, b)).  No array: the GPU engine's kernel keeps
// no per-lane path buffer in scratch.
template <class F>
SIM_HDI uint32_t icnt_route(const SimCfg& c, uint32_t a, uint32_t b, F&& emit) {
  const uint32_t k = c.topo_k ? c.topo_k : 2, n = c.topo_n ? c.topo_n : 1;
  uint32_t m = 0;
  switch (c.topo) {
    case TOPO_FLY: {  // destination-tag routing, most significant digit first
      const uint64_t kn1 = ipow(k, n - 1);
      uint64_t cur = a;
      for (uint32_t s = 0; s < n && m < (uint32_t)kMaxPathLinks; ++s) {
        const uint64_t pw = ipow(k, n - 1 - s);             // weight of the digit this stage sets
        const uint32_t port = (uint32_t)((b / pw) % k);
        const uint64_t r = (cur / (pw * k)) * pw + cur % pw;  // the router: cur without that digit
        emit((uint32_t)(((uint64_t)s * kn1 + r) * k + port));
        ++m;
        cur = cur - ((cur / pw) % k) * pw + (uint64_t)port * pw;
      }
      return m;
    }
    case TOPO_CMESH:
    case TOPO_MESH:
    case TOPO_TORUS: {  // dimension-order routing on a k-ary n-cube
      const uint32_t conc = c.topo == TOPO_CMESH ? (c.topo_conc ? c.topo_conc : 1) : 1;
      const uint32_t P = 2 * n + conc;
      uint64_t cur = a / conc;
      const uint64_t dst = b / conc;
      uint64_t pw = 1;
      for (uint32_t d = 0; d < n; ++d, pw *= k) {
        for (uint32_t guard = 0; guard < k && m + 1 < (uint32_t)kMaxPathLinks; ++guard) {
          const uint32_t x = (uint32_t)((cur / pw) % k), y = (uint32_t)((dst / pw) % k);
          if (x == y) break;
          bool up = y > x;
          if (c.topo == TOPO_TORUS) {
            const uint32_t fwd = (y + k - x) % k;  // hops going up (with wrap)
            up = fwd <= k - fwd;
          }
          emit((uint32_t)(cur * P + 2 * d + (up ? 0 : 1)));
          ++m;
          const uint32_t nx = up ? (x + 1) % k : (x + k - 1) % k;
          cur = cur - (uint64_t)x * pw + (uint64_t)nx * pw;
        }
      }
      emit((uint32_t)(cur * P + 2 * n + b % conc));
      ++m;
      return m;
    }
    case TOPO_FATTREE: {  // up to the lowest common ancestor (d-mod-k), then down
      const uint64_t kn = ipow(k, n);
      uint32_t lvl = 1;
      {
        uint64_t x = a / k, y = b / k;
        while (x != y && lvl < n) {
          x /= k;
          y /= k;
          ++lvl;
        }
      }
      // the level-l switch on the way up holds the source's digits above l
      // and the destination's below l (d-mod-k took digit i at level i); its
      // up port is the destination's digit l.  On the way down every switch
      // and port is the destination's: one down link per (level, destination)
      for (uint32_t l = 0; l + 1 < lvl; ++l) {
        const uint64_t pk = ipow(k, l + 1);
        emit((uint32_t)((uint64_t)l * kn + (a / pk) * pk + b % pk));
        ++m;
      }
      for (uint32_t l = lvl - 1; l-- > 0;) {
        emit((uint32_t)((uint64_t)n * kn + (uint64_t)l * kn + b % kn));
        ++m;
      }
      emit((uint32_t)(2ull * n * kn + b % kn));
      ++m;
      return m;
    }
    default: {  // flattened butterfly: one hop per differing dimension between routers
      // (node / conc; the config check guarantees k^n * conc >= nodes, so every
      // router index is < k^n and every link index < icnt_link_count)
      const uint32_t conc = c.topo_conc ? c.topo_conc : 1;
      const uint32_t P = n * k + conc;
      uint64_t cur = a / conc, pw = 1;
      const uint64_t dst = b / conc;
      for (uint32_t d = 0; d < n; ++d, pw *= k) {
        const uint32_t x = (uint32_t)((cur / pw) % k), y = (uint32_t)((dst / pw) % k);
        if (x == y) continue;
        emit((uint32_t)(cur * P + d * k + y));
        ++m;
        cur = cur - (uint64_t)x * pw + (uint64_t)y * pw;
      }
      emit((uint32_t)(cur * P + n * k + b % conc));
      ++m;
      return m;
    }
  }
}

// reserve the route of one packet (a -> b, uncontended arrival p.t) and
// return its extra delay (fs)
SIM_HDI uint64_t icnt_reserve(const SimCfg& c, Pkt& p, uint32_t a, uint32_t b, uint64_t* link_free) {
  const uint32_t nl = icnt_routers(c, a, b);  // one link per router crossed (icnt_route)
  const uint64_t nflits = (p.size + c.flit_size - 1) / c.flit_size;
  const uint64_t occ = (nflits ? nflits : 1) * c.per_icnt;
  const uint64_t hop = ((uint64_t)c.hop_icnt + c.chan_icnt) * c.per_icnt, last = (uint64_t)c.chan_icnt * c.per_icnt;
  uint64_t D = 0;
  uint32_t h = 0;
  icnt_route(c, a, b, [&](uint32_t l) {
#if !defined(__HIP_DEVICE_COMPILE__) && !defined(NDEBUG)
    if (l >= icnt_link_count(c)) throw std::logic_error("icnt_reserve: link index outside the topology");
#endif
    // uncontended departure onto link h (the route's schedule ends at p.t)
    const uint64_t back = (uint64_t)(nl - 1 - (h < nl ? h : nl - 1)) * hop + last;
    const uint64_t d = p.t > back ? p.t - back : 0;
    uint64_t t = d + D;
    const uint64_t f = link_free[l];
    if (f > t) {
      D += f - t;
      t = f;
    }
    link_free[l] = t + occ;
    ++h;
  });
  p.t += D;
  return D;
}

// the epoch-boundary pass over this epoch's outboxes (requests [sub][sm][cap],
// replies [sm][sub][cap]); `refs` holds up to every cell x cap entries, stat
// accumulates {delayed packets, delay in interconnect cycles}; a packet's
// reference is (cell << 16 | index): cells and cell capacities < 2^16
// (icnt_contention_fits)
template <class P>
SIM_HDI void icnt_contend(const SimCfg& c, Pkt* box_req, const uint32_t* cnt_req, uint32_t cap_req, Pkt* box_rep,
                          const uint32_t* cnt_rep, uint32_t cap_rep, uint64_t* link_free, uint32_t* refs,
                          uint64_t* stat) {
  const uint32_t ncell = c.n_sm * c.n_subpart;
  const uint32_t cpc = c.cores_per_cluster ? c.cores_per_cluster : 1;
  for (int dir = 0; dir < 2; ++dir) {
    const uint32_t* cnt = dir == 0 ? cnt_req : cnt_rep;
    // every packet of the epoch in cell order: (cell << 16 | index in the cell)
    const uint32_t total = P::scan((int)ncell, [&](int i) -> uint32_t { return cnt[i]; },
                                   [&](int i, uint32_t off) {
                                     for (uint32_t j = 0; j < cnt[i]; ++j) refs[off + j] = (uint32_t)i << 16 | j;
                                   });
    P::sync();
    if (total == 0) continue;
    P::one([&] {
      uint64_t delayed = 0, wait = 0;
      for (uint32_t r = 0; r < total; ++r) {
        const uint32_t cell = refs[r] >> 16, j = refs[r] & 0xffffu;
        uint32_t a, b;
        Pkt* p;
        if (dir == 0) {  // request: SM (cell % n_sm) -> sub-partition (cell / n_sm)
          a = (cell % c.n_sm) / cpc;
          b = c.n_clusters + cell / c.n_sm;
          p = &box_req[(uint64_t)cell * cap_req + j];
        } else {  // reply: sub-partition (cell % n_subpart) -> SM (cell / n_subpart)
          a = c.n_clusters + cell % c.n_subpart;
          b = (cell / c.n_subpart) / cpc;
          p = &box_rep[(uint64_t)cell * cap_rep + j];
        }
        const uint64_t D = icnt_reserve(c, *p, a, b, link_free);
        if (D) {
          ++delayed;
          wait += fdiv(D, c.dv_icnt);
        }
      }
      stat[0] += delayed;
      stat[1] += wait;
    });
    P::sync();
  }
}

}  // namespace asim
