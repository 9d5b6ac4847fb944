// Trace residency windows shared by the engines (host code).
//
// A kernel's decoded trace (instructions, coalesced accesses, per-warp
// streams) is either resident whole, or -- when it is larger than the window
// -- streamed per CTA: the engine keeps rings holding about W x the
// resident-CTA capacity of the kernel (index = global index & (cap - 1);
// the access ring has kMaxAccess mirrored entries so an instruction's
// accesses are always contiguous), and before every run the window follows
// the dispatch cursor: CTAs every SM is done with are dropped, CTAs the next
// epochs' dispatch can reach are brought in (epoch_decide's refill stop
// guarantees a run never dispatches past the resident ones).
//
// The source of a window is the host ReadyKernel.  When that is itself
// streamed (-trace_host_budget_mb: csrc/trace/trace.h KernelReader), only
// the CTAs of the window are held on the host too, parsed from the trace
// file as the window advances: host memory is proportional to the resident
// CTAs, not to the kernel (the reference streams thread blocks from the
// file, gpu-simulator/trace-parser/trace_parser.cc:387-447).
//
// `Mem` says where the rings live: device memory (GPU engine: hipMalloc +
// hipMemcpy) or host memory (CPU engine: plain copies; a whole host-resident
// kernel is used in place).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "../model/epoch.h"
#include "../trace/trace.h"

namespace asim {

// what a window needs to know about the dispatch state: the replicated
// cursors (SM 0's copy) and every SM's resident CTAs
struct DispatchView {
  uint32_t k_uid[kMaxConc] = {};
  uint32_t next_cta[kMaxConc] = {};
  uint32_t next_ctax[kMaxConc][kMaxXcd] = {};
  struct Sm {
    uint32_t cta_id[kMaxCta];
    uint8_t cta_valid[kMaxCta];
    uint8_t cta_ks[kMaxCta];
  };
  std::vector<Sm> sms;
};

template <class Mem>
class TraceWindows {
 public:
  struct Slot {
    void* insts = nullptr;
    void* accs = nullptr;
    void* streams = nullptr;
    size_t cap_insts = 0, cap_accs = 0, cap_streams = 0;
    ReadyKernel* rk = nullptr;
    bool streamed = false;
    bool in_place = false;            // whole host kernel used where it is (host rings)
    uint64_t w_ctas = 0;              // window target in CTAs
    uint32_t lo = 0, avail = 0;       // resident CTAs [lo, avail)
    uint64_t icap = 0, acap = 0, ccap = 0;  // ring entries (powers of two)
    std::vector<uint32_t> ib, ab;     // whole host kernels: per-CTA first instruction / access index (+ end)
  };
  Mem mem;
  Slot s[kMaxConc];
  uint64_t resident_peak = 0, refills = 0;

  ~TraceWindows() { release(); }
  void release() {
    for (Slot& b : s) {
      if (!b.in_place) {
        mem.free(b.insts);
        mem.free(b.accs);
        mem.free(b.streams);
      }
      b = Slot{};
    }
  }

  // per-CTA first instruction / access index of CTA c (the end marks at n_cta)
  uint64_t ib(const Slot& b, uint32_t c) const {
    return b.rk->streamed() ? b.rk->ib[c - b.rk->cta_lo] : b.ib[c];
  }
  uint64_t ab(const Slot& b, uint32_t c) const {
    return b.rk->streamed() ? b.rk->ab[c - b.rk->cta_lo] : b.ab[c];
  }
  // host CTAs [lo, hi) available to read (a streamed host kernel parses on)
  void host_resident(Slot& b, uint32_t lo, uint32_t hi) {
    if (b.rk->streamed()) b.rk->resident(lo, hi);
  }

  void launch(uint32_t slot, ReadyKernel& k, KernelDesc& d, const SimCfg& c) {
    Slot& b = s[slot];
    b.rk = &k;
    b.streamed = plan(b, k, d, c);
    if (b.streamed) {
      fill(slot, d, 0, std::min<uint32_t>(d.n_cta, (uint32_t)b.w_ctas), true);
    } else if (Mem::kHost) {
      // the whole kernel, in place
      if (!b.in_place) {
        mem.free(b.insts);
        mem.free(b.accs);
        mem.free(b.streams);
      }
      b.in_place = true;
      b.insts = (void*)k.insts.data();
      b.accs = (void*)k.accs.data();
      b.streams = (void*)k.streams.data();
      b.cap_insts = b.cap_accs = b.cap_streams = 0;
      d.insts = k.insts.data();
      d.accs = k.accs.data();
      d.streams = k.streams.data();
      d.imask = d.amask = d.cmask = ~0u;
      d.cta_avail = d.n_cta;
    } else {
      upload(b.insts, b.cap_insts, k.insts.data(), k.insts.size() * sizeof(TInst));
      upload(b.accs, b.cap_accs, k.accs.data(), k.accs.size() * sizeof(TAcc));  // may be empty
      upload(b.streams, b.cap_streams, k.streams.data(), k.streams.size() * sizeof(WStream));
      d.insts = reinterpret_cast<const TInst*>(b.insts);
      d.accs = reinterpret_cast<const TAcc*>(b.accs);
      d.streams = reinterpret_cast<const WStream*>(b.streams);
      d.imask = d.amask = d.cmask = ~0u;
      d.cta_avail = d.n_cta;
    }
    note();
  }
  void done(uint32_t slot) { s[slot].rk = nullptr; }

  // before every engine run: for each streamed running kernel, drop the CTAs
  // every SM is done with and bring in up to the window past the dispatch
  // cursor, so the next epochs' dispatch (epoch.h dispatch_bound) finds them
  // resident.  `read(view)` fills the dispatch state (called only when a
  // kernel streams).
  template <class Read>
  void ensure(KernelTab& kt, const SimCfg& c, Read&& read) {
    uint32_t streamed = 0;
    for (uint32_t k = 0; k < (uint32_t)kMaxConc; ++k)
      if ((kt.active >> k & 1u) && s[k].rk && s[k].streamed && kt.k[k].cta_avail < kt.k[k].n_cta) streamed |= 1u << k;
    if (!streamed) return;
    DispatchView v;
    read(v);
    for (uint32_t sl = 0; sl < (uint32_t)kMaxConc; ++sl) {
      if (!(streamed >> sl & 1u)) continue;
      KernelDesc& kd = kt.k[sl];
      Slot& b = s[sl];
      const bool fresh = v.k_uid[sl] != kd.uid;  // not dispatched from yet (cursors reset at its first epoch)
      const uint32_t nx0 = fresh ? 0u : v.next_cta[sl];
      uint32_t nxx[kMaxXcd] = {};
      if (!fresh)
        for (int xi = 0; xi < kMaxXcd; ++xi) nxx[xi] = v.next_ctax[sl][xi];
      // lowest CTA still needed: resident on an SM, or the first undispatched
      uint64_t lo = kd.n_cta;
      if (c.n_xcd > 1) {
        for (uint32_t xi = 0; xi < c.n_xcd; ++xi) {
          const uint64_t ncx = kd.n_cta > xi ? (kd.n_cta - xi + c.n_xcd - 1) / c.n_xcd : 0;
          if (nxx[xi] < ncx) lo = std::min<uint64_t>(lo, xi + (uint64_t)c.n_xcd * nxx[xi]);
        }
      } else {
        lo = std::min<uint64_t>(lo, nx0);
      }
      if (!fresh)
        for (const DispatchView::Sm& m : v.sms)
          for (int i = 0; i < kMaxCta; ++i)
            if (m.cta_valid[i] && m.cta_ks[i] == sl) lo = std::min<uint64_t>(lo, m.cta_id[i]);
      const uint64_t bound = dispatch_bound(c, kd, nx0, nxx);
      const uint32_t need = (uint32_t)std::min<uint64_t>(kd.n_cta, bound + 1);
      if (need <= b.avail && lo >= b.lo) continue;  // the window still covers the next epochs
      const uint32_t lo32 = (uint32_t)std::min<uint64_t>(lo, need);
      // aim a whole window past the oldest CTA still needed, at least `need`,
      // shrunk to what the rings hold (they grow only when `need` does not fit)
      uint32_t hi = (uint32_t)std::min<uint64_t>(kd.n_cta, std::max<uint64_t>(need, lo32 + b.w_ctas));
      host_resident(b, lo32, hi);
      auto fits = [&](uint32_t h) {
        return h - lo32 <= b.ccap && ib(b, h) - ib(b, lo32) <= b.icap && ab(b, h) - ab(b, lo32) <= b.acap;
      };
      if (fits(need)) {
        uint32_t a = need, e = hi;  // largest fitting end in [need, hi]
        while (a < e) {
          const uint32_t m = a + (e - a + 1) / 2;
          if (fits(m)) a = m;
          else e = m - 1;
        }
        hi = a;
      } else {
        hi = need;
      }
      const bool overlap = lo32 >= b.lo && lo32 <= b.avail;
      fill(sl, kd, lo32, hi, !overlap);
    }
  }

  bool any_streamed() const {
    for (const Slot& b : s)
      if (b.rk && b.streamed) return true;
    return false;
  }
  uint64_t resident_bytes() const {
    uint64_t t = 0;
    for (const Slot& b : s) t += b.cap_insts + b.cap_accs + b.cap_streams;
    return t;
  }

 private:
  static uint64_t pow2ceil(uint64_t v) {
    uint64_t p = 1;
    while (p < v) p <<= 1;
    return p;
  }
  void note() { resident_peak = std::max(resident_peak, resident_bytes()); }

  void upload(void*& d, size_t& cap, const void* h, size_t bytes) {
    if (bytes > cap || !d) {
      mem.free(d);
      cap = bytes + bytes / 4 + 4096;
      d = mem.alloc(cap);
    }
    if (bytes && h) mem.write(d, h, bytes);
  }

  // Streaming plan of a kernel (-gpu_trace_window / -sim_trace_window):
  // per-CTA first instruction / access index, ring capacities.  A whole host
  // kernel streams only when its CTAs occupy ascending, non-overlapping
  // ranges (every loader here writes them so) and it is larger than the
  // window; a streamed host kernel always streams.
  bool plan(Slot& b, ReadyKernel& k, const KernelDesc& kd, const SimCfg& c) {
    const uint64_t cpc = std::max<uint64_t>(1, std::min<uint32_t>(kd.cta_per_sm, kMaxCta));
    // window in CTAs: -gpu_trace_window x the kernel's resident-CTA capacity;
    // a host-streamed kernel always has one (2 x when the option is 0)
    const uint64_t w = (uint64_t)(c.trace_window ? c.trace_window : 2) * c.n_sm * cpc;
    if (!k.streamed() && (Mem::kHost || !c.trace_window || w >= kd.n_cta || !k.warps_per_cta)) return false;
    const uint32_t n = kd.n_cta;
    if (!k.streamed()) {
      const uint32_t wpc = k.warps_per_cta;
      b.ib.assign((size_t)n + 1, 0);
      b.ab.assign((size_t)n + 1, 0);
      uint64_t hi_i = 0, hi_a = 0;
      for (uint32_t cc = 0; cc < n; ++cc) {
        uint64_t ilo = ~0ull, ihi = 0, alo = ~0ull, ahi = 0;
        for (uint32_t wi = 0; wi < wpc; ++wi) {
          const WStream& ws = k.streams[(size_t)cc * wpc + wi];
          if (!ws.count) continue;
          ilo = std::min<uint64_t>(ilo, ws.begin);
          ihi = std::max<uint64_t>(ihi, (uint64_t)ws.begin + ws.count);
          for (uint32_t j = ws.begin; j < ws.begin + ws.count; ++j) {
            const TInst& in = k.insts[j];
            if (in.space == S_SHARED || !in.width || in.mem == kNoMem) continue;
            alo = std::min<uint64_t>(alo, in.mem);
            ahi = std::max<uint64_t>(ahi, (uint64_t)in.mem + std::min<uint32_t>(in.width, kMaxAccess));
          }
        }
        if (ilo == ~0ull) ilo = ihi = hi_i;
        if (alo == ~0ull) alo = ahi = hi_a;
        if (ilo < hi_i || alo < hi_a) return false;  // not CTA-ordered: keep the whole kernel
        b.ib[cc] = (uint32_t)ilo;
        b.ab[cc] = (uint32_t)alo;
        hi_i = ihi;
        hi_a = ahi;
      }
      b.ib[n] = (uint32_t)hi_i;
      b.ab[n] = (uint32_t)hi_a;
    }
    b.w_ctas = w;
    const uint32_t we = (uint32_t)std::min<uint64_t>(n, w);
    host_resident(b, 0, we);
    b.ccap = pow2ceil(w);
    b.icap = pow2ceil(std::max<uint64_t>(1, ib(b, we) - ib(b, 0)));
    b.acap = pow2ceil(std::max<uint64_t>(1, ab(b, we) - ab(b, 0)));
    b.lo = b.avail = 0;
    if (b.in_place) {  // the slot's previous kernel was used in place: nothing to free
      b.insts = b.accs = b.streams = nullptr;
      b.cap_insts = b.cap_accs = b.cap_streams = 0;
      b.in_place = false;
    }
    return true;
  }

  // copy global elements [first, first + count) of an array whose element
  // `base` is at src[0] into a ring of `cap` entries (+ `pad` mirrored
  // leading entries) at index & (cap - 1)
  void ring_write(void* ring, size_t esz, uint64_t cap, uint64_t pad, const void* src, uint64_t base, uint64_t first,
                  uint64_t count) {
    char* r = static_cast<char*>(ring);
    const char* p = static_cast<const char*>(src) + (first - base) * esz;
    while (count) {
      const uint64_t q = first & (cap - 1);
      const uint64_t n = std::min<uint64_t>(count, cap - q);
      mem.write(r + q * esz, p, n * esz);
      if (q < pad) mem.write(r + (cap + q) * esz, p, std::min<uint64_t>(n, pad - q) * esz);
      p += n * esz;
      first += n;
      count -= n;
    }
  }

  // make CTAs [lo, hi) of slot `slot` resident (growing the rings when the
  // range does not fit); `full`: rewrite the whole range, else append
  // [avail, hi)
  void fill(uint32_t slot, KernelDesc& d, uint32_t lo, uint32_t hi, bool full) {
    Slot& b = s[slot];
    ReadyKernel& k = *b.rk;
    const uint32_t wpc = k.warps_per_cta;
    host_resident(b, lo, hi);
    while (hi - lo > b.ccap) { b.ccap <<= 1; full = true; }
    while (ib(b, hi) - ib(b, lo) > b.icap) { b.icap <<= 1; full = true; }
    while (ab(b, hi) - ab(b, lo) > b.acap) { b.acap <<= 1; full = true; }
    if (k.streamed() && (b.icap > kStreamInstMask + 1 || b.acap > kStreamAccMask + 1))
      throw std::runtime_error("host-streamed trace window exceeds 2^28 instructions / 2^31 accesses");
    auto ensure_cap = [&](void*& p, size_t& cap, size_t bytes) {
      if (p && cap >= bytes) return;
      mem.free(p);
      cap = bytes;
      p = mem.alloc(cap);
    };
    ensure_cap(b.insts, b.cap_insts, b.icap * sizeof(TInst));
    ensure_cap(b.accs, b.cap_accs, (b.acap + kMaxAccess) * sizeof(TAcc));
    ensure_cap(b.streams, b.cap_streams, b.ccap * wpc * sizeof(WStream));
    const uint32_t from = full ? lo : std::max(lo, b.avail);
    if (hi > from) {
      const uint64_t i0 = ib(b, from), i1 = ib(b, hi), a0 = ab(b, from), a1 = ab(b, hi);
      ring_write(b.insts, sizeof(TInst), b.icap, 0, k.insts.data(), k.streamed() ? k.ibase : 0, i0, i1 - i0);
      if (a1 > a0)
        ring_write(b.accs, sizeof(TAcc), b.acap, kMaxAccess, k.accs.data(), k.streamed() ? k.abase : 0, a0, a1 - a0);
      ring_write(b.streams, sizeof(WStream) * wpc, b.ccap, 0, k.streams.data(), k.streamed() ? k.cta_lo : 0, from,
                 hi - from);
    }
    b.lo = lo;
    b.avail = hi;
    ++refills;
    d.insts = reinterpret_cast<const TInst*>(b.insts);
    d.accs = reinterpret_cast<const TAcc*>(b.accs);
    d.streams = reinterpret_cast<const WStream*>(b.streams);
    d.imask = (uint32_t)(b.icap - 1);
    d.amask = (uint32_t)(b.acap - 1);
    d.cmask = (uint32_t)(b.ccap - 1);
    d.cta_avail = hi;
    note();
  }
};

}  // namespace asim
