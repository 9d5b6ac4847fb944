// Address decoding and set-index hashing (host + device).
//
// Semantics follow the reference address decoder (addrdec.cc:95-201,
// partition_address :78-93) and cache set-index functions
// (gpu-cache.cc:80-153).  IPOLY is implemented generically as GF(2)
// polynomial reduction -- index ^ ((h(x) * x^n) mod P(x)) -- which reproduces
// the reference's hand-expanded IPOLY(5)/IPOLY(37)/IPOLY(67) tables
// (hashing.cc:9-97) for 16/32/64 banks and extends to other power-of-two
// bank counts.  The reference's RANDOM mode keeps a rand()-filled hash map
// (addrdec.cc:164-185); here it is a stateless splitmix hash so the CPU and GPU
// engines (and every rank) agree without shared state.
#pragma once
#include "config.h"

namespace asim {

struct AddrTlx {
  uint32_t chip;
  uint32_t bk;
  uint32_t row;
  uint32_t col;
  uint32_t burst;
  uint32_t sub;  // global sub-partition id
};

SIM_HDI uint64_t pack_bits(uint64_t mask, uint64_t val, int high, int low) {
  uint64_t r = 0;
  int pos = 0;
  uint64_t m = mask;
  // iterate set bits of the mask in [low, high)
  while (m) {
    int i = __builtin_ctzll(m);
    m &= m - 1;
    if (i < low) continue;
    if (i >= high) break;
    r |= ((val >> i) & 1ull) << pos;
    ++pos;
  }
  return r;
}

SIM_HDI int ilog2u(uint64_t x) { return x ? 63 - __builtin_clzll(x) : 0; }

// runs of a gather mask restricted to bit positions [low, high) (host side,
// once per configuration): the decoder then costs a few shifts per run
// instead of a loop over every mask bit
SIM_HDI BitRuns make_runs(uint64_t mask, int high, int low) {
  BitRuns r{};
  if (high < 64) mask &= (1ull << high) - 1;
  if (low > 0) mask &= ~((1ull << low) - 1);
  int pos = 0;
  while (mask) {
    const int sh = __builtin_ctzll(mask);
    const uint64_t m = mask >> sh;
    const int w = (~m == 0) ? 64 - sh : __builtin_ctzll(~m);
    if (r.n == 8) { r.n = 0xff; return r; }
    r.sh[r.n] = (uint8_t)sh;
    r.w[r.n] = (uint8_t)w;
    r.out[r.n] = (uint8_t)pos;
    ++r.n;
    pos += w;
    mask = (w + sh >= 64) ? 0 : (mask & ~(((w >= 64) ? ~0ull : ((1ull << w) - 1)) << sh));
  }
  return r;
}
SIM_HDI uint64_t run_gather(const BitRuns& r, uint64_t v) {
  uint64_t o = 0;
  for (int i = 0; i < (int)r.n && i < 8; ++i) {
    const uint64_t m = r.w[i] >= 64 ? ~0ull : ((1ull << r.w[i]) - 1);
    o |= ((v >> r.sh[i]) & m) << r.out[i];
  }
  return o;
}

// GF(2): (h * x^n) mod P, P given with its x^n term (bit n set).
SIM_HDI uint32_t gf2_mulxn_mod(uint64_t h, int n, uint32_t poly) {
  // linear in h: XOR over the set bits i of h of x^(i+n) mod P, walking the
  // powers of x only as far as h's highest set bit
  uint32_t xp = 1;
  for (int i = 0; i < n; ++i) {
    xp <<= 1;
    if (xp >> n & 1u) xp ^= poly;
  }
  uint32_t r = 0;
  for (; h; h >>= 1) {
    if (h & 1ull) r ^= xp;
    xp <<= 1;
    if (xp >> n & 1u) xp ^= poly;
  }
  return r;
}

// primitive polynomials (bit n included) and the number of high address bits
// folded in; rows 4..6 reproduce IPOLY(5/37/67) of the reference.
SIM_HDI uint32_t ipoly_poly(int n) {
  switch (n) {
    case 1: return 0x3;
    case 2: return 0x7;
    case 3: return 0xB;
    case 4: return 0x13;   // x^4+x+1
    case 5: return 0x25;   // x^5+x^2+1
    case 6: return 0x43;   // x^6+x+1
    case 7: return 0x83;   // x^7+x+1
    case 8: return 0x11D;  // x^8+x^4+x^3+x^2+1
    case 9: return 0x211;
    case 10: return 0x409;
    default: return 0x43;
  }
}
SIM_HDI int ipoly_hbits(int n) {
  switch (n) {
    case 4: return 13;
    case 5: return 15;
    case 6: return 19;
    default: return 3 * n + 1;
  }
}
SIM_HDI uint32_t ipoly_hash(uint64_t higher, uint32_t index, uint32_t nbanks) {
  int n = ilog2u(nbanks);
  if (n == 0) return 0;
  int hb = ipoly_hbits(n);
  uint64_t h = hb >= 64 ? higher : (higher & ((1ull << hb) - 1));
  return (index ^ gf2_mulxn_mod(h, n, ipoly_poly(n))) & (nbanks - 1);
}
SIM_HDI uint32_t bitwise_hash(uint64_t higher, uint32_t index, uint32_t nbanks) {
  return (index ^ (uint32_t)(higher & (nbanks - 1))) & (nbanks - 1);
}
SIM_HDI uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

SIM_HDI AddrTlx addr_decode(const SimCfg& c, uint64_t addr) {
  AddrTlx t;
  uint64_t rest_high;
  const uint32_t nsub = c.n_sub_per_mem;
  auto field = [&](int f, uint64_t v) -> uint32_t {
    return c.addr_runs[f].n != 0xff ? (uint32_t)run_gather(c.addr_runs[f], v)
                                    : (uint32_t)pack_bits(c.addr_mask[f], v, c.mk_hi[f], c.mk_lo[f]);
  };
  if (!c.gap) {
    t.chip = field(AF_CHIP, addr);
    t.bk = field(AF_BK, addr);
    t.row = field(AF_ROW, addr);
    t.col = field(AF_COL, addr);
    t.burst = field(AF_BURST, addr);
    rest_high = addr >> (c.addr_chip_s + c.log2ch + c.log2sub);
  } else {
    uint64_t hi = addr >> c.addr_chip_s;
    uint64_t rest = ((hi / c.n_mem) << c.addr_chip_s) | (addr & ((1ull << c.addr_chip_s) - 1));
    rest_high = hi / c.n_mem;
    t.chip = (uint32_t)(hi % c.n_mem);
    t.bk = field(AF_BK, rest);
    t.row = field(AF_ROW, rest);
    t.col = field(AF_COL, rest);
    t.burst = field(AF_BURST, rest);
  }
  switch (c.part_index) {
    case PIDX_BITWISE:
      t.chip = bitwise_hash(rest_high, t.chip, c.n_mem);
      break;
    case PIDX_IPOLY:
    case PIDX_PAE: {  // PAE has no decoder case in the reference (defect D11): use IPOLY
      uint32_t sp = (t.chip << c.log2sub) + (t.bk & (nsub - 1));
      sp = ipoly_hash(rest_high, sp, c.n_ch_pow2 * nsub);
      if (c.gap) sp = sp % (c.n_mem * nsub);
      t.chip = sp >> c.log2sub;  // sub-partitions per channel: a power of two
      t.sub = sp;
      return t;
    }
    case PIDX_RANDOM: {
      uint64_t ca = addr >> (c.addr_chip_s - c.log2sub);
      uint32_t id = (uint32_t)(splitmix64(ca) % (c.n_mem * nsub));
      t.chip = id >> c.log2sub;
      t.sub = id;
      return t;
    }
    default:
      break;
  }
  if (t.chip >= c.n_mem) t.chip %= c.n_mem;
  t.sub = (t.chip << c.log2sub) + (t.bk & (nsub - 1));
  return t;
}

// address with the channel / sub-partition selection bits squeezed out
// (used for L2 set indexing, reference partition_address addrdec.cc:78-93)
SIM_HDI uint64_t partition_address(const SimCfg& c, uint64_t addr) {
  if (!c.gap)
    return c.part_runs.n != 0xff ? run_gather(c.part_runs, addr)
                                 : pack_bits(~(c.addr_mask[AF_CHIP] | c.sub_id_mask), addr, 64, 0);
  uint64_t pa = ((addr >> c.addr_chip_s) / c.n_mem) << c.addr_chip_s;
  pa |= addr & ((1ull << c.addr_chip_s) - 1);
  return c.part_runs.n != 0xff ? run_gather(c.part_runs, pa) : pack_bits(~c.sub_id_mask, pa, 64, 0);
}

// XCD-private L2s (SimCfg::n_xcd): the destination sub-partition of a request
// from SM `sm` whose address decodes to the global sub-partition `gsub`: the
// slice of the SM's own XCD picked by the address's low slice bits
SIM_HDI uint32_t l2_slice_of(const SimCfg& c, uint32_t sm, uint32_t gsub) {
  if (!c.n_xcd) return gsub;
  return ((sm % c.n_xcd) << c.log2_spx) | (gsub & ((1u << c.log2_spx) - 1u));
}
// set-index address of an XCD slice (and of the MALL behind it): the
// slice-select bits squeezed out of the channel field
SIM_HDI uint64_t xcd_partition_address(const SimCfg& c, uint64_t a) {
  const uint32_t lo = (uint32_t)c.addr_chip_s, k = c.log2_spx;
  return ((a >> (lo + k)) << lo) | (a & ((1ull << lo) - 1));
}

SIM_HDI uint32_t cache_set_index(const CacheGeom& g, uint64_t addr) {
  const int lb = ilog2u(g.line);
  const int sb = ilog2u(g.nsets);
  const uint32_t idx = (uint32_t)((addr >> lb) & (g.nsets - 1));
  switch (g.set_index) {
    case SIDX_FERMI: {
      if (g.nsets != 32 && g.nsets != 64) return idx;
      uint32_t lower = (uint32_t)((addr >> lb) & 0x1F);
      uint32_t upper = (uint32_t)((addr & 0xE000) >> 13);
      upper |= (uint32_t)((addr & 0x20000) >> 14);
      upper |= (uint32_t)((addr & 0x80000) >> 15);
      uint32_t s = lower ^ upper;
      if (g.nsets == 64) s |= (uint32_t)((addr & 0x1000) >> 7);
      return s & (g.nsets - 1);
    }
    case SIDX_BITWISE_XOR:
      return bitwise_hash(addr >> (lb + sb), idx, g.nsets);
    case SIDX_HASH_IPOLY:
      return ipoly_hash(addr >> (lb + sb), idx, g.nsets);
    default:
      return idx;
  }
}

}  // namespace asim
