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

// GF(2): (h * x^n) mod P, P given with its x^n term (bit n set).
SIM_HDI uint32_t gf2_mulxn_mod(uint64_t h, int n, uint32_t poly) {
  // process bits of h from the top: r = r*x + bit, reduced, then * x^n
  uint32_t r = 0;
  for (int i = 63; i >= 0; --i) {
    r = (r << 1) | (uint32_t)((h >> i) & 1ull);
    if (r >> n & 1u) r ^= poly;
  }
  for (int i = 0; i < n; ++i) {
    r <<= 1;
    if (r >> n & 1u) r ^= poly;
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
  if (!c.gap) {
    t.chip = (uint32_t)pack_bits(c.addr_mask[AF_CHIP], addr, c.mk_hi[AF_CHIP], c.mk_lo[AF_CHIP]);
    t.bk = (uint32_t)pack_bits(c.addr_mask[AF_BK], addr, c.mk_hi[AF_BK], c.mk_lo[AF_BK]);
    t.row = (uint32_t)pack_bits(c.addr_mask[AF_ROW], addr, c.mk_hi[AF_ROW], c.mk_lo[AF_ROW]);
    t.col = (uint32_t)pack_bits(c.addr_mask[AF_COL], addr, c.mk_hi[AF_COL], c.mk_lo[AF_COL]);
    t.burst = (uint32_t)pack_bits(c.addr_mask[AF_BURST], addr, c.mk_hi[AF_BURST], c.mk_lo[AF_BURST]);
    rest_high = addr >> (c.addr_chip_s + c.log2ch + c.log2sub);
  } else {
    uint64_t hi = addr >> c.addr_chip_s;
    uint64_t rest = ((hi / c.n_mem) << c.addr_chip_s) | (addr & ((1ull << c.addr_chip_s) - 1));
    rest_high = hi / c.n_mem;
    t.chip = (uint32_t)(hi % c.n_mem);
    t.bk = (uint32_t)pack_bits(c.addr_mask[AF_BK], rest, c.mk_hi[AF_BK], c.mk_lo[AF_BK]);
    t.row = (uint32_t)pack_bits(c.addr_mask[AF_ROW], rest, c.mk_hi[AF_ROW], c.mk_lo[AF_ROW]);
    t.col = (uint32_t)pack_bits(c.addr_mask[AF_COL], rest, c.mk_hi[AF_COL], c.mk_lo[AF_COL]);
    t.burst = (uint32_t)pack_bits(c.addr_mask[AF_BURST], rest, c.mk_hi[AF_BURST], c.mk_lo[AF_BURST]);
  }
  switch (c.part_index) {
    case PIDX_BITWISE:
      t.chip = bitwise_hash(rest_high, t.chip, c.n_mem);
      break;
    case PIDX_IPOLY:
    case PIDX_PAE: {  // PAE has no decoder case in the reference (defect D11): use IPOLY
      uint32_t sp = t.chip * nsub + (t.bk & (nsub - 1));
      sp = ipoly_hash(rest_high, sp, c.n_ch_pow2 * nsub);
      if (c.gap) sp = sp % (c.n_mem * nsub);
      t.chip = sp / nsub;
      t.sub = sp;
      return t;
    }
    case PIDX_RANDOM: {
      uint64_t ca = addr >> (c.addr_chip_s - c.log2sub);
      uint32_t id = (uint32_t)(splitmix64(ca) % (c.n_mem * nsub));
      t.chip = id / nsub;
      t.sub = id;
      return t;
    }
    default:
      break;
  }
  if (t.chip >= c.n_mem) t.chip %= c.n_mem;
  t.sub = t.chip * nsub + (t.bk & (nsub - 1));
  return t;
}

// address with the channel / sub-partition selection bits squeezed out
// (used for L2 set indexing, reference partition_address addrdec.cc:78-93)
SIM_HDI uint64_t partition_address(const SimCfg& c, uint64_t addr) {
  if (!c.gap) return pack_bits(~(c.addr_mask[AF_CHIP] | c.sub_id_mask), addr, 64, 0);
  uint64_t pa = ((addr >> c.addr_chip_s) / c.n_mem) << c.addr_chip_s;
  pa |= addr & ((1ull << c.addr_chip_s) - 1);
  return pack_bits(~c.sub_id_mask, pa, 64, 0);
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
