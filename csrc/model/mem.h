// Memory partition model: one DRAM channel with its L2 sub-partitions.
//
// Reference: memory_partition_unit / memory_sub_partition (l2cache.h:72,160;
// l2cache.cc:305-375 dram_cycle, :463-595 cache_cycle with the ROP delay
// queue), dram_t (dram.cc:289-682) and the FR-FCFS scheduler
// (dram_sched.cc:109-258).  Re-designed as fixed-capacity rings and flat
// associative tables so that one wavefront owns one channel on the GPU; the
// per-domain clocks are integer femtoseconds and are stepped in time order
// inside each PDES epoch (reference next_clock_domain, gpu-sim.cc:1833-1854).
#pragma once
#include "sm.h"

namespace asim {

struct L2Line {
  uint64_t tag;
  uint32_t lru;
  uint8_t valid;  // sector mask
  uint8_t dirty;  // sector mask
  uint8_t pad[2];
};

struct L2Mshr {
  uint64_t line;
  uint8_t requested;
  uint8_t valid;
  uint8_t merges;
  uint8_t pad[5];
};

struct L2Wait {  // request waiting for sectors from DRAM
  uint64_t line;
  uint32_t tag;
  uint16_t src;
  uint8_t need;     // sectors still missing
  uint8_t sectors;  // sectors requested (reply payload)
  uint8_t type;     // request packet type
  uint8_t valid;
  uint8_t pad[6];
};

struct DramReq {
  uint64_t line;     // line address
  uint64_t ready;    // fs: leaves the L2->DRAM latency pipe
  uint32_t row;
  uint16_t bank;
  uint8_t sector;    // sector index 0..3
  uint8_t write;
  uint8_t sub;       // local sub-partition index
  uint8_t pad[7];
};

struct DramRet {
  uint64_t line;
  uint64_t ready;    // fs
  uint8_t sector;
  uint8_t sub;
  uint8_t pad[6];
};

struct DramBank {
  uint64_t t_col_ok;   // dram cycles
  uint64_t t_pre_ok;
  uint64_t t_act_ok;
  uint32_t row;
  uint8_t open;
  uint8_t pad[3];
};

enum L2StatType : uint8_t { L2T_RD = 0, L2T_WR, L2T_ATOM, L2T_COUNT };
enum L2StatOut : uint8_t { L2O_HIT = 0, L2O_MISS, L2O_MSHR_HIT, L2O_RES_FAIL, L2O_COUNT };
struct MemStats {
  uint64_t l2[L2T_COUNT][L2O_COUNT];
  uint64_t dram_rd;
  uint64_t dram_wr;
  uint64_t dram_act;
  uint64_t dram_pre;
  uint64_t dram_busy_cycles;   // cycles with a column command in flight on the bus
  uint64_t dram_cycles;
  uint64_t dram_q_occ;         // sum of queue occupancy per dram cycle
  uint64_t l2_cycles;
  uint64_t l2_busy;            // L2 cycles that processed a request
  uint64_t rop_occ;
  uint64_t pkts_in;
  uint64_t pkts_out;
  uint64_t bytes_in;
  uint64_t bytes_out;
  uint64_t l2_evict_dirty;
  uint64_t icnt_stall;
  uint64_t icnt_backlog;       // arrivals that waited in the input backlog (sum over epochs of its length)
  uint64_t icnt_ovf_drop;      // arrivals lost to a full backlog ring (must stay 0)
  uint64_t icnt_conflicts;     // request net: ready inputs not granted by this output port (per cycle)
  uint64_t icnt_queue_cycles;  // request net: icnt cycles granted packets waited at this output port
  uint64_t icnt_arb_cycles;    // request net: icnt cycles with at least one input ready
  // below the L2 (per 32 B sector): what leaves the L2 for memory (the
  // Infinity Fabric traffic rocprofv3 counts as TCC_EA0_RDREQ / WRREQ), and
  // how the memory-attached cache (MALL) in front of DRAM served it
  uint64_t l2_mem_rd, l2_mem_wr;
  // the same traffic in requests (a line fill, a write packet or a line
  // write-back is one request, of 32-128 B): rocprofv3 TCC_EA0_RDREQ / WRREQ
  uint64_t l2_mem_rd_req, l2_mem_wr_req;
  uint64_t mall_rd_hit, mall_rd_miss, mall_wr, mall_wb;
  uint64_t icnt_inj_stall;  // icnt cycles a ready reply waited for room in the router's injection queue
};

struct SubPart {
  Pkt inq[kMemInQ];   // arrivals sorted by time
  uint32_t inq_head, inq_n;
  Pkt rop[kRopQ];     // ROP delay queue (p.t = exit time)
  uint32_t rop_head, rop_n;
  Pkt reply[kReplyQ];
  uint32_t rep_head, rep_n;
  uint64_t port_free;  // fs
  DramRet fill[64];    // DRAM -> L2 queue
  uint32_t fill_head, fill_n;
  uint32_t l2_stamp;
  uint32_t n_wait;
  uint32_t n_l2dram;   // requests of this sub in the L2->DRAM path
  uint32_t ovf_head, ovf_n;  // arrival backlog ring (MemCtx::ovf) for arrivals that did not fit in inq
  uint16_t arb_next, arb_cnt;  // crossbar output-port arbiter: next input, grants left at the pointer
  int64_t inj_allow0;  // -icnt_link_contention 2: reply flits the node's injection queue takes at the epoch start
  uint64_t inj_used;   // ... and the reply flits injected since
  L2Mshr mshr[kMaxL2Mshr];
  L2Wait wait[kMaxL2Wait];
  MemStats st;
};

struct alignas(16) ChanState {
  uint32_t id;
  uint32_t pub_nz;    // bit p: the reply cells of mailbox parity p were last written with packets
  uint64_t t_icnt;    // next tick time of each domain (fs)
  uint64_t t_l2;
  uint64_t t_dram;
  uint64_t dcycle;    // dram cycle counter
  uint64_t min_emit;  // earliest arrival time (fs) of the replies injected this epoch
  uint64_t inj_t0_fs; // start of the epoch (fs): the reply injection back-pressure's reference
  // DRAM
  DramReq lat[kDramLat];  // L2 -> DRAM latency pipe (FIFO)
  uint32_t lat_head, lat_n;
  DramReq q[kDramQ];    // scheduler queue (pool; age order via q_age)
  uint32_t q_n;
  uint16_t qw_n;        // writes among them (separate write queue accounting)
  uint8_t wmode;        // write-drain mode of the separate write queue
  uint8_t pad1;
  DramBank bk[kMaxBanksDram];
  uint64_t t_rrd_ok, t_ccd_ok, t_rd_ok, t_wr_ok, bus_free;
  uint64_t t_ccdl_ok[8];
  DramRet ret[kDramRet];
  uint32_t ret_head, ret_n;
  uint64_t q_seq;        // arrival sequence for FR-FCFS age order
  // MALL: read hits on their way back to the L2 (DRAM returns use ret[])
  DramRet mret[kMallRet];
  uint32_t mret_head, mret_n;
  uint32_t mall_stamp;
  uint32_t q_hi;  // DRAM queue slots in use lie below q_hi (dram_enqueue takes the lowest free slot)
  uint64_t q_age[kDramQ];
  uint8_t q_valid[kDramQ];
  uint16_t ocnt[kMaxSubPerCh][kMaxSmTot];  // replies put in each (dst SM) cell this epoch
  uint64_t skey[kMemInQ];                  // gather scratch: sort keys
  uint32_t sref[kMemInQ];                  // gather scratch: (src << 16 | k)
  uint32_t srank[kMemInQ > kMaxSmTot ? kMemInQ : kMaxSmTot];  // gather scratch: ranks / per-source offsets
  SubPart sp[kMaxSubPerCh];
  // L2 tag arrays of the channel's sub-partitions, one pool: sub-partition j
  // owns lines [j * sets * assoc, (j + 1) * sets * assoc), so a channel with
  // one sub-partition can hold twice the lines of one with two (MI355X: 4 MiB
  // per XCD = 16 channels x 2048 lines of 128 B)
  L2Line l2[kMaxL2LinesCh];
};
SIM_HDI L2Line* l2_tags(ChanState& ch, const SimCfg& c, uint32_t sub) {
  return ch.l2 + (size_t)sub * c.l2.nsets * c.l2.assoc;
}

SIM_HDI uint32_t sp_out_count(const ChanState& ch, uint32_t sub, uint32_t dst) { return ch.ocnt[sub][dst]; }
SIM_HDI void sp_out_count_inc(ChanState& ch, uint32_t sub, uint32_t dst) { ch.ocnt[sub][dst]++; }

struct MemCtx {
  const SimCfg* cfg;
  Pkt* outbox;          // this epoch's reply outbox base: [dst_sm][src_sub][cap]
  uint32_t* outcnt;     // [dst_sm][src_sub]
  uint32_t out_cap;
  uint32_t n_src_sub;   // row stride (number of sub-partitions)
  uint64_t win_end;     // fs, exclusive
  Pkt* ovf;             // per-sub-partition arrival backlog rings [n_subpart][ovf_cap] (global memory)
  uint32_t ovf_cap;
  L2Line* mall;         // this channel's MALL lines [mall_sets][mall_assoc] (global memory), nullptr = no MALL
  const uint64_t* rt_st = nullptr;  // -icnt_link_contention 2: the router model's state (injection back-pressure)
};

// ---------------------------------------------------------------------------
SIM_HDI uint32_t dram_bank_of(const SimCfg& c, const AddrTlx& t) { return t.bk % (c.nbk ? c.nbk : 1); }
SIM_HDI uint32_t dram_bkgrp(const SimCfg& c, uint32_t bank) {
  uint32_t ng = c.nbkgrp ? c.nbkgrp : 1;
  if (c.bkgrp_index_policy == 1) return bank % ng;  // lower bits
  uint32_t per = c.nbk / ng ? c.nbk / ng : 1;
  return (bank / per) % ng;
}

// Requests between the L2 and the DRAM data return hold channel credits
// (reference memory_partition_unit arbitration: a private credit per
// sub-partition + a shared pool of sched_queue + return_queue entries,
// l2cache.cc:120-140, borrowed when a request enters the DRAM latency queue);
// the per-sub-partition share also bounds what one L2 slice can queue.
SIM_HDI bool l2dram_can(const ChanState& ch, const SubPart& sp, const SimCfg& c, uint32_t n) {
  return sp.n_l2dram + n <= c.q_l2_dram && ch.lat_n + ch.q_n + n <= c.dram_credits &&
         ch.lat_n + n <= (uint32_t)kDramLat;
}

// write requests to the fabric are at most 64 B: one per half line with data
SIM_HDI uint32_t wr_requests(uint32_t sectors) { return ((sectors & 3u) ? 1u : 0u) + ((sectors & 12u) ? 1u : 0u); }

SIM_HDI void l2dram_push(ChanState& ch, SubPart& sp, const SimCfg& c, uint32_t sub, uint64_t line,
                         uint32_t sector, bool write, uint64_t now_fs) {
  DramReq& r = ch.lat[(ch.lat_head + ch.lat_n) % kDramLat];
  AddrTlx t = addr_decode(c, line + sector * 32ull);
  r.line = line;
  r.ready = now_fs + (uint64_t)c.dram_latency * c.per_l2;
  r.row = t.row;
  r.bank = (uint16_t)dram_bank_of(c, t);
  r.sector = (uint8_t)sector;
  r.write = write ? 1 : 0;
  r.sub = (uint8_t)sub;
  ch.lat_n++;
  sp.n_l2dram++;
  if (write) sp.st.l2_mem_wr++;
  else sp.st.l2_mem_rd++;
}

// ---- MALL (memory-attached last-level cache) -------------------------------
constexpr uint8_t kSubNone = 0xff;  // DramReq::sub of a MALL write-back (holds no L2 credit)
SIM_HDI uint32_t mall_set(const SimCfg& c, uint64_t line) {
  const uint64_t a = c.n_xcd ? xcd_partition_address(c, line) : partition_address(c, line);
  return (uint32_t)((a >> 7) & (c.mall_sets - 1));
}
template <class P>
SIM_HDI int mall_find(const L2Line* b, uint32_t assoc, uint64_t line) {
  const uint64_t m = P::ballot((int)assoc, [&](int w) { return b[w].valid && b[w].tag == line; });
  return m ? ffs64(m) : -1;
}
template <class P>
SIM_HDI int mall_victim(const L2Line* b, uint32_t assoc) {
  return P::argmin((int)assoc, [&](int w) -> uint64_t { return b[w].valid ? ((1ull << 40) | b[w].lru) : (uint64_t)w; });
}
// a MALL line lives in global memory: one lane stores it, the fence orders it
// before the wave's next probe
template <class P>
SIM_HDI void mall_put(L2Line* b, int w, const L2Line& v) {
  P::one([&] { b[w] = v; });
  P::sync();
}
// room in the DRAM scheduler for n more requests of one kind
SIM_HDI bool dram_room(const ChanState& ch, const SimCfg& c, bool write, uint32_t n) {
  const uint32_t qcap = amin<uint32_t>(c.dram_queue ? c.dram_queue : 1, kDramQ);
  if (ch.q_n + n > (uint32_t)kDramQ) return false;
  if (!c.wq_enable) return ch.q_n + n <= qcap;
  return write ? ch.qw_n + n <= c.wq_size : ch.q_n - ch.qw_n + n <= qcap;
}
template <class P>
SIM_HDI void dram_enqueue(ChanState& ch, const DramReq& h) {
  const int f = P::find_first(kDramQ, [&](int i) -> bool { return !ch.q_valid[i]; });
  if (f < 0) return;  // (dram_room is checked first: never full here)
  ch.qw_n += h.write ? 1 : 0;
  ch.q[f] = h;
  ch.q_valid[f] = 1;
  if ((uint32_t)f + 1u > ch.q_hi) ch.q_hi = (uint32_t)f + 1u;
  ch.q_age[f] = ch.q_seq++;
  ch.q_n++;
}
// dirty sectors of a MALL victim go to DRAM (false: no room, nothing changed)
template <class P>
SIM_HDI bool mall_writeback(ChanState& ch, const SimCfg& c, const L2Line& v, uint64_t now_fs) {
  if (!(v.valid && v.dirty)) return true;
  const uint32_t n = (uint32_t)popc64(v.dirty);
  if (!dram_room(ch, c, true, n)) return false;
  for (uint32_t s = 0; s < 4; ++s) {
    if (!(v.dirty >> s & 1u)) continue;
    DramReq r;
    const AddrTlx t = addr_decode(c, v.tag + s * 32ull);
    r.line = v.tag;
    r.ready = now_fs;
    r.row = t.row;
    r.bank = (uint16_t)dram_bank_of(c, t);
    r.sector = (uint8_t)s;
    r.write = 1;
    r.sub = kSubNone;
    dram_enqueue<P>(ch, r);
  }
  ch.sp[0].st.mall_wb += n;
  return true;
}
// install sector `sec` of `line` (a DRAM read returning or a write absorbed);
// false: the victim's write-back found no room (the caller decides)
template <class P>
SIM_HDI bool mall_install(ChanState& ch, const SimCfg& c, L2Line* b, uint64_t line, uint32_t sec, bool dirty,
                          uint64_t now_fs) {
  int w = mall_find<P>(b, c.mall_assoc, line);
  L2Line v;
  if (w < 0) {
    w = mall_victim<P>(b, c.mall_assoc);
    const L2Line old = P::uni(b[w]);
    if (!mall_writeback<P>(ch, c, old, now_fs)) return false;
    v.tag = line;
    v.valid = 0;
    v.dirty = 0;
    v.pad[0] = v.pad[1] = 0;
  } else {
    v = P::uni(b[w]);
  }
  v.valid |= (uint8_t)(1u << sec);
  if (dirty) v.dirty |= (uint8_t)(1u << sec);
  v.lru = ++ch.mall_stamp;
  mall_put<P>(b, w, v);
  return true;
}

// ---- L2 tag array (lane-parallel over ways) ----
template <class P>
SIM_HDI int l2_find(const L2Line* T, const CacheGeom& g, uint32_t set, uint64_t line) {
  const L2Line* b = &T[set * g.assoc];
  for (uint32_t o = 0; o < g.assoc; o += 64) {
    int n = (int)amin<uint32_t>(64, g.assoc - o);
    uint64_t m = P::ballot(n, [&](int w) { return b[o + w].valid && b[o + w].tag == line; });
    if (m) return (int)o + ffs64(m);
  }
  return -1;
}
template <class P>
SIM_HDI int l2_victim(const L2Line* T, const CacheGeom& g, uint32_t set) {
  const L2Line* b = &T[set * g.assoc];
  return P::argmin((int)g.assoc, [&](int w) -> uint64_t {
    return b[w].valid ? ((1ull << 40) | b[w].lru) : (uint64_t)w;
  });
}
SIM_HDI uint32_t l2_set(const SimCfg& c, uint64_t line) {
  return cache_set_index(c.l2, c.n_xcd ? xcd_partition_address(c, line) : partition_address(c, line));
}

// allocate a line for `line` (evicting, writing back dirty sectors);
// returns way or -1 if the write-back cannot be queued
template <class P>
SIM_HDI int l2_alloc(ChanState& ch, SubPart& sp, const SimCfg& c, uint32_t sub, uint32_t set,
                     uint64_t line, uint64_t now_fs) {
  const CacheGeom& g = c.l2;
  L2Line* T = l2_tags(ch, c, sub);
  int v = l2_victim<P>(T, g, set);
  L2Line& L = T[set * g.assoc + v];
  if (L.valid && L.dirty) {
    uint32_t nd = (uint32_t)popc64(L.dirty);
    if (!l2dram_can(ch, sp, c, nd)) return -1;
    for (uint32_t s = 0; s < 4; ++s)
      if (L.dirty >> s & 1u) l2dram_push(ch, sp, c, sub, L.tag, s, true, now_fs);
    sp.st.l2_evict_dirty++;
    sp.st.l2_mem_wr_req += wr_requests(L.dirty);
  }
  L.tag = line;
  L.valid = 0;
  L.dirty = 0;
  L.lru = ++sp.l2_stamp;
  return v;
}

SIM_HDI bool reply_push(SubPart& sp, uint8_t type, const Pkt& req, uint8_t sectors) {
  if (sp.rep_n >= (uint32_t)kReplyQ) return false;
  Pkt& r = sp.reply[(sp.rep_head + sp.rep_n) % kReplyQ];
  r.addr = req.addr;
  r.t = 0;
  r.tag = req.tag;
  r.src = req.dst;  // sub-partition id
  r.dst = req.src;  // requesting SM
  r.type = type;
  r.sectors = sectors;
  r.size = (type == P_WR_ACK) ? 8 : (uint16_t)(8 + 32 * popc64(sectors));
  r.aux = 0;
  sp.rep_n++;
  return true;
}

// process the request at the head of the ROP queue; false = stalled
template <class P>
SIM_HDI bool l2_access(ChanState& ch, SubPart& sp, const SimCfg& c, uint32_t sub, const Pkt& p,
                       uint64_t now_fs) {
  const CacheGeom& g = c.l2;
  const uint32_t set = l2_set(c, p.addr);
  const uint32_t stype = p.type == P_WR ? L2T_WR : (p.type == P_ATOM ? L2T_ATOM : L2T_RD);
  if (sp.rep_n >= (uint32_t)kReplyQ) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
  // MEMORY_SUBPARTITION_UNIT trace: outcome 0 hit, 1 miss, 2 mshr hit, 3 write-through
  auto trace = [&](uint16_t outcome) {
    if (trace_mem_on(c, TS_MEMORY_SUBPARTITION_UNIT, ch.id))
      P::one([&] { trace_put(c, c.n_sm + ch.id, fdiv(now_fs, c.dv_l2), EV_L2_ACCESS, (uint16_t)(sub << 8 | outcome), p.addr); });
  };
  L2Line* T = l2_tags(ch, c, sub);
  int way = g.disabled ? -1 : l2_find<P>(T, g, set, p.addr);
  if (p.type == P_WR) {
    if (g.disabled || g.wpolicy == WP_WRITE_THROUGH) {
      uint32_t n = (uint32_t)popc64(p.sectors);
      if (!l2dram_can(ch, sp, c, n)) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
      for (uint32_t s = 0; s < 4; ++s)
        if (p.sectors >> s & 1u) l2dram_push(ch, sp, c, sub, p.addr, s, true, now_fs);
      sp.st.l2_mem_wr_req += wr_requests(p.sectors);
      if (way >= 0) T[set * g.assoc + way].valid |= p.sectors;
      trace(3);
    } else {
      // write-back L2 (reference data_cache wr_hit_wb / wr_miss_*,
      // gpu-cache.cc:1229-1599): a hit, or any write-allocate miss, makes
      // the sectors dirty; only whole-sector writes are readable at once
      // (lazy fetch on read); 'N' sends a miss to DRAM without allocating
      const uint8_t have = way >= 0 ? T[set * g.assoc + way].valid : (uint8_t)0;
      const bool hit = way >= 0 && (have & p.sectors) == p.sectors;
      const uint32_t bytes = p.size > 8 ? p.size - 8u : 0u;
      const bool full = bytes >= 32u * (uint32_t)popc64(p.sectors);
      const uint8_t wa = g.walloc;
      if (!hit && wa == 'N') {
        const uint32_t n = (uint32_t)popc64(p.sectors);
        if (!l2dram_can(ch, sp, c, n)) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
        for (uint32_t s2 = 0; s2 < 4; ++s2)
          if (p.sectors >> s2 & 1u) l2dram_push(ch, sp, c, sub, p.addr, s2, true, now_fs);
        sp.st.l2_mem_wr_req += wr_requests(p.sectors);
        sp.st.l2[stype][L2O_MISS]++;
        trace(1);
        reply_push(sp, P_WR_ACK, p, p.sectors);
        return true;
      }
      // fetch-on-write ('F', partial sectors) and naive ('W') read the
      // written sectors that are not yet readable
      const bool fetch = !hit && (wa == 'W' || (wa == 'F' && !full));
      int mi = -1, mfree = 0;
      uint8_t rd = 0;
      const int nm = (int)amin<uint32_t>(g.mshr_entries, kMaxL2Mshr);
      if (fetch) {
        mi = P::find_first(nm, [&](int i) -> bool { return sp.mshr[i].valid && sp.mshr[i].line == p.addr; });
        if (mi < 0) mfree = P::find_first(nm, [&](int i) -> bool { return !sp.mshr[i].valid; });
        rd = p.sectors & (uint8_t)~have;
        if (mi >= 0) rd &= (uint8_t)~sp.mshr[mi].requested;
        if (mfree < 0 || !l2dram_can(ch, sp, c, (uint32_t)popc64(rd))) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
      }
      if (way < 0) {
        way = l2_alloc<P>(ch, sp, c, sub, set, p.addr, now_fs);
        if (way < 0) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
      }
      if (hit) {
        sp.st.l2[stype][L2O_HIT]++;
        trace(0);
      } else {
        sp.st.l2[stype][L2O_MISS]++;
        trace(1);
      }
      L2Line& L = T[set * g.assoc + way];
      if (full && !fetch) L.valid |= p.sectors;
      L.dirty |= p.sectors;
      if (g.repl == REPL_LRU) L.lru = ++sp.l2_stamp;
      if (fetch && rd) {
        if (mi < 0) {
          mi = mfree;
          sp.mshr[mi].valid = 1;
          sp.mshr[mi].line = p.addr;
          sp.mshr[mi].requested = 0;
          sp.mshr[mi].merges = 0;
        }
        sp.mshr[mi].requested |= rd;
        for (uint32_t s2 = 0; s2 < 4; ++s2)
          if (rd >> s2 & 1u) l2dram_push(ch, sp, c, sub, p.addr, s2, false, now_fs);
        sp.st.l2_mem_rd_req++;
      }
    }
    reply_push(sp, P_WR_ACK, p, p.sectors);
    return true;
  }
  // read / atomic
  uint8_t have = way >= 0 ? T[set * g.assoc + way].valid : 0;
  uint8_t miss = p.sectors & (uint8_t)~have;
  const uint8_t rtype = p.type == P_ATOM ? P_ATOM_REPLY : P_RD_REPLY;
  if (miss == 0) {
    L2Line& L = T[set * g.assoc + way];
    if (g.repl == REPL_LRU) L.lru = ++sp.l2_stamp;
    if (p.type == P_ATOM) L.dirty |= p.sectors;
    reply_push(sp, rtype, p, p.sectors);
    sp.st.l2[stype][L2O_HIT]++;
    trace(0);
    return true;
  }
  if (sp.n_wait >= (uint32_t)kMaxL2Wait) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
  const int nm = (int)amin<uint32_t>(g.mshr_entries, kMaxL2Mshr);
  int mi = P::find_first(nm, [&](int i) -> bool { return sp.mshr[i].valid && sp.mshr[i].line == p.addr; });
  // a sectored L2 ('S') fetches the missing sectors it was asked for; a
  // line-granular one ('N', e.g. the MI355X L2: TCC_EA0_RDREQ_128B dominates
  // its fills) fetches every sector of the line it does not hold
  const uint8_t fetch = g.sectored ? miss : (uint8_t)(0xFu & ~have);
  uint8_t need_req = mi >= 0 ? (uint8_t)(fetch & ~sp.mshr[mi].requested) : fetch;
  if (need_req == 0) {
    if (sp.mshr[mi].merges >= g.mshr_merge) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
    sp.mshr[mi].merges++;
    sp.st.l2[stype][L2O_MSHR_HIT]++;
    trace(2);
  } else {
    uint32_t nreq = (uint32_t)popc64(need_req);
    if (!l2dram_can(ch, sp, c, nreq)) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
    if (mi < 0) {
      mi = P::find_first(nm, [&](int i) -> bool { return !sp.mshr[i].valid; });
      if (mi < 0) { sp.st.l2[stype][L2O_RES_FAIL]++; return false; }
      sp.mshr[mi].valid = 1;
      sp.mshr[mi].line = p.addr;
      sp.mshr[mi].requested = 0;
      sp.mshr[mi].merges = 0;
    }
    sp.mshr[mi].requested |= need_req;
    for (uint32_t s = 0; s < 4; ++s)
      if (need_req >> s & 1u) l2dram_push(ch, sp, c, sub, p.addr, s, false, now_fs);
    sp.st.l2_mem_rd_req++;
    sp.st.l2[stype][L2O_MISS]++;
    trace(1);
  }
  // waiter entry (first free)
  uint32_t wi = sp.n_wait;
  for (uint32_t b = 0; b < sp.n_wait; b += 64) {
    int n = (int)amin<uint32_t>(64, sp.n_wait - b);
    uint64_t m = P::ballot(n, [&](int i) { return !sp.wait[b + i].valid; });
    if (m) { wi = b + ffs64(m); break; }
  }
  L2Wait& e = sp.wait[wi];
  e.line = p.addr;
  e.tag = p.tag;
  e.src = p.src;
  e.need = miss;
  e.sectors = p.sectors;
  e.type = p.type;
  e.valid = 1;
  if (wi == sp.n_wait) sp.n_wait++;
  return true;
}

// DRAM data for one sector returns to the L2
template <class P>
SIM_HDI bool l2_fill(ChanState& ch, SubPart& sp, const SimCfg& c, uint32_t sub, const DramRet& r,
                     uint64_t now_fs) {
  const CacheGeom& g = c.l2;
  L2Line* T = l2_tags(ch, c, sub);
  const uint8_t sbit = (uint8_t)(1u << r.sector);
  // replies this fill will generate must fit
  uint32_t nrep = 0;
  for (uint32_t b = 0; b < sp.n_wait; b += 64) {
    int n = (int)amin<uint32_t>(64, sp.n_wait - b);
    uint64_t m = P::ballot(n, [&](int i) {
      const L2Wait& e = sp.wait[b + i];
      return e.valid && e.line == r.line && e.need == sbit;
    });
    nrep += (uint32_t)popc64(m);
  }
  if (sp.rep_n + nrep > (uint32_t)kReplyQ) return false;
  if (!g.disabled) {
    uint32_t set = l2_set(c, r.line);
    int way = l2_find<P>(T, g, set, r.line);
    if (way < 0) {
      way = l2_alloc<P>(ch, sp, c, sub, set, r.line, now_fs);
      if (way < 0) return false;
    }
    L2Line& L = T[set * g.assoc + way];
    L.valid |= sbit;
    if (g.repl == REPL_LRU) L.lru = ++sp.l2_stamp;
  }
  const int nm = (int)amin<uint32_t>(g.mshr_entries, kMaxL2Mshr);
  int mi = P::find_first(nm, [&](int i) -> bool { return sp.mshr[i].valid && sp.mshr[i].line == r.line; });
  if (mi >= 0) {
    sp.mshr[mi].requested &= (uint8_t)~sbit;
    if (!sp.mshr[mi].requested) sp.mshr[mi].valid = 0;
  }
  for (uint32_t b = 0; b < sp.n_wait; b += 64) {
    int n = (int)amin<uint32_t>(64, sp.n_wait - b);
    uint64_t m = P::ballot(n, [&](int i) {
      const L2Wait& e = sp.wait[b + i];
      return e.valid && e.line == r.line && (e.need & sbit);
    });
    while (m) {
      int i = ffs64(m);
      m &= m - 1;
      L2Wait& e = sp.wait[b + i];
      e.need &= (uint8_t)~sbit;
      if (e.need) continue;
      Pkt q;
      q.addr = e.line;
      q.tag = e.tag;
      q.src = e.src;
      q.dst = (uint16_t)(ch.id * c.n_sub_per_mem + sub);
      q.type = e.type;
      q.sectors = e.sectors;
      q.size = 0;
      q.t = 0;
      q.aux = 0;
      reply_push(sp, e.type == P_ATOM ? P_ATOM_REPLY : P_RD_REPLY, q, e.sectors);
      if (e.type == P_ATOM && !g.disabled) {
        uint32_t set = l2_set(c, r.line);
        int way = l2_find<P>(T, g, set, r.line);
        if (way >= 0) T[set * g.assoc + way].dirty |= e.sectors;
      }
      e.valid = 0;
    }
  }
  while (sp.n_wait && !sp.wait[sp.n_wait - 1].valid) sp.n_wait--;
  return true;
}

// one L2 cycle of one sub-partition
template <class P>
SIM_HDI void l2_cycle(ChanState& ch, SubPart& sp, const SimCfg& c, uint32_t sub, uint64_t now_fs) {
  sp.st.l2_cycles++;
  sp.st.rop_occ += sp.rop_n;
  if (sp.fill_n) {
    const DramRet& r = sp.fill[sp.fill_head];
    if (r.ready <= now_fs) {
      DramRet rr = r;
      if (l2_fill<P>(ch, sp, c, sub, rr, now_fs)) {
        sp.fill_head = (sp.fill_head + 1) % 64;
        sp.fill_n--;
      }
    }
  }
  if (sp.rop_n) {
    const Pkt& p = sp.rop[sp.rop_head];
    if (p.t <= now_fs) {
      Pkt pp = p;
      if (l2_access<P>(ch, sp, c, sub, pp, now_fs)) {
        sp.rop_head = (sp.rop_head + 1) % kRopQ;
        sp.rop_n--;
        sp.st.l2_busy++;
      }
    }
  }
}

// one interconnect cycle of one sub-partition: accept an arrival into the
// ROP queue and start injecting a reply
template <class P>
SIM_HDI void mem_icnt_cycle(ChanState& ch, SubPart& sp, const SimCfg& c, const MemCtx& x,
                            uint32_t sub, uint64_t now_fs) {
  if (sp.inq_n && sp.rop_n < (uint32_t)kRopQ && sp.rop_n < c.q_icnt_l2 + c.rop_latency &&
      sp.inq[sp.inq_head].t <= now_fs) {
    // the output port grants one ready input per cycle
    XbarGrant g = xbar_pick<P>(sp.inq, sp.inq_head, sp.inq_n, kMemInQ, now_fs, c, fdiv(now_fs, c.dv_icnt),
                               sp.arb_next, sp.arb_cnt, c.n_sm);
    sp.st.icnt_arb_cycles++;
    sp.st.icnt_conflicts += g.ready - 1;
    {
      Pkt p = xbar_take(sp.inq, sp.inq_head, sp.inq_n, kMemInQ, g.off);
      sp.st.icnt_queue_cycles += fdiv(now_fs - p.t, c.dv_icnt);
      p.t = now_fs + (uint64_t)c.rop_latency * c.per_l2;
      sp.rop[(sp.rop_head + sp.rop_n) % kRopQ] = p;
      sp.rop_n++;
      sp.st.pkts_in++;
      sp.st.bytes_in += p.size;
    }
  }
  if (sp.rep_n && sp.port_free <= now_fs) {
    Pkt r = sp.reply[sp.rep_head];
    uint32_t nflits = (r.size + c.flit_size - 1) / c.flit_size;
    if (c.link_contention == 2 && !rt_inj_ok(c, ch.inj_t0_fs, sp.inj_allow0, sp.inj_used, nflits, now_fs)) {
      sp.st.icnt_inj_stall++;  // the node's injection queue is full
      return;
    }
    if (c.link_contention == 2) sp.inj_used += nflits;
    uint64_t done = now_fs + (uint64_t)(nflits - 1) * c.per_icnt;
    {  // serialisation may run past the window end (see sm_inject)
      uint32_t gsub = ch.id * c.n_sub_per_mem + sub;
      uint32_t cell = (uint32_t)r.dst * x.n_src_sub + gsub;
      // per-destination counter kept in the reply's own slot count array
      uint32_t n = sp_out_count(ch, sub, r.dst);
      if (n < x.out_cap) {
        r.t = done + icnt_pkt_lat_fs(c, r.dst, gsub);
        ch.min_emit = amin(ch.min_emit, r.t);
        P::one([&] { x.outbox[(uint64_t)cell * x.out_cap + n] = r; });
        sp_out_count_inc(ch, sub, r.dst);
        sp.rep_head = (sp.rep_head + 1) % kReplyQ;
        sp.rep_n--;
        sp.port_free = now_fs + (uint64_t)nflits * c.per_icnt;
        sp.st.pkts_out++;
        sp.st.bytes_out += r.size;
      } else {
        sp.st.icnt_stall++;
      }
    }
  }
}

}  // namespace asim

namespace asim {

// ---------------------------------------------------------------------------
// DRAM channel: one DRAM clock.  FR-FCFS (row hits first, then oldest) with
// per-bank ACT/PRE state machines and HBM-style dual command bus
// (reference dram_t::cycle dram.cc:289-552, frfcfs dram_sched.cc:109-258).
template <class P>
SIM_HDI void dram_cycle(ChanState& ch, const SimCfg& c, const MemCtx& x, uint64_t now_fs) {
  MemStats& st = ch.sp[0].st;
  const uint64_t t = ch.dcycle++;
  st.dram_cycles++;
  // latency pipe -> (MALL) -> scheduler queue
  while (ch.lat_n) {
    const DramReq h = ch.lat[ch.lat_head];
    if (h.ready > now_fs) break;
    if (x.mall) {
      L2Line* b = x.mall + (uint64_t)mall_set(c, h.line) * c.mall_assoc;
      if (h.write) {
        // write-back, write-allocate: the MALL absorbs the sector
        if (!mall_install<P>(ch, c, b, h.line, h.sector, true, now_fs)) break;
        st.mall_wr++;
        ch.sp[h.sub].n_l2dram--;
        ch.lat_head = (ch.lat_head + 1) % kDramLat;
        ch.lat_n--;
        continue;
      }
      const int w = mall_find<P>(b, c.mall_assoc, h.line);
      if (w >= 0 && (P::uni(b[w].valid) >> h.sector & 1u)) {
        if (ch.mret_n >= (uint32_t)kMallRet) break;
        DramRet& o = ch.mret[(ch.mret_head + ch.mret_n) % kMallRet];
        o.line = h.line;
        o.sector = h.sector;
        o.sub = h.sub;
        o.ready = now_fs;
        ch.mret_n++;
        L2Line v = P::uni(b[w]);
        v.lru = ++ch.mall_stamp;
        mall_put<P>(b, w, v);
        st.mall_rd_hit++;
        ch.sp[h.sub].n_l2dram--;
        ch.lat_head = (ch.lat_head + 1) % kDramLat;
        ch.lat_n--;
        continue;
      }
    }
    // reads and writes have their own capacity with a separate write queue
    // (reference dram_t::full, dram.cc:160-175)
    if (!dram_room(ch, c, h.write != 0, 1)) break;
    if (x.mall) st.mall_rd_miss++;
    dram_enqueue<P>(ch, h);
    ch.lat_head = (ch.lat_head + 1) % kDramLat;
    ch.lat_n--;
  }
  // MALL hits, then DRAM data returns -> DRAM->L2 queues
  const uint32_t fcap = amin<uint32_t>(c.q_dram_l2 ? c.q_dram_l2 : 1, 64);
  while (ch.mret_n) {
    const DramRet& r = ch.mret[ch.mret_head];
    if (r.ready > now_fs) break;
    SubPart& sp = ch.sp[r.sub];
    if (sp.fill_n >= fcap) break;
    sp.fill[(sp.fill_head + sp.fill_n) % 64] = r;
    sp.fill_n++;
    ch.mret_head = (ch.mret_head + 1) % kMallRet;
    ch.mret_n--;
  }
  while (ch.ret_n) {
    const DramRet& r = ch.ret[ch.ret_head];
    if (r.ready > now_fs) break;
    SubPart& sp = ch.sp[r.sub];
    if (sp.fill_n >= fcap) break;
    // a read that missed the MALL allocates there on its way back (a dirty
    // victim without DRAM queue room leaves the line uncached instead)
    if (x.mall) {
      L2Line* b = x.mall + (uint64_t)mall_set(c, r.line) * c.mall_assoc;
      (void)mall_install<P>(ch, c, b, r.line, r.sector, false, now_fs);
    }
    sp.fill[(sp.fill_head + sp.fill_n) % 64] = r;
    sp.fill_n++;
    ch.ret_head = (ch.ret_head + 1) % kDramRet;
    ch.ret_n--;
  }
  st.dram_q_occ += ch.q_n;
  if (ch.q_n == 0) return;
  // the scans visit the slots in use only (the empty ones above never qualify)
  const int qn = (int)ch.q_hi;
  const uint32_t burst = amax<uint32_t>(1, c.BL / (c.data_cmd_ratio ? c.data_cmd_ratio : 1));
  if (c.simple_dram) {
    // oldest request, one column access per DRAM cycle, no bank state
    int o = P::argmin(qn, [&](int i) -> uint64_t { return ch.q_valid[i] ? ch.q_age[i] : ~0ull; });
    if (o < 0 || t < ch.t_ccd_ok) return;
    const DramReq r = ch.q[o];
    if (!r.write) {
      if (ch.ret_n >= (uint32_t)kDramRet) return;
      DramRet& d = ch.ret[(ch.ret_head + ch.ret_n) % kDramRet];
      d.line = r.line;
      d.sector = r.sector;
      d.sub = r.sub;
      d.ready = (t + burst) * c.per_dram + (x.mall ? c.mall_miss_fs : 0);
      ch.ret_n++;
      st.dram_rd++;
    } else {
      st.dram_wr++;
    }
    ch.t_ccd_ok = t + burst;
    st.dram_busy_cycles += burst;
    ch.q_valid[o] = 0;
    while (ch.q_hi && !ch.q_valid[ch.q_hi - 1]) --ch.q_hi;
    ch.q_n--;
    ch.qw_n -= r.write ? 1 : 0;
    if (r.sub != kSubNone) ch.sp[r.sub].n_l2dram--;
    return;
  }
  // separate write queue: serve reads until the writes reach the high
  // watermark, then drain writes down to the low watermark (reference
  // frfcfs_scheduler::schedule, dram_sched.cc:118-130).  With no read queued
  // at all the writes are served too, so a kernel's tail cannot strand them.
  uint32_t only = 2;  // 0 reads only, 1 writes only, 2 both
  if (c.wq_enable) {
    if (!ch.wmode && ch.qw_n >= c.wq_hi) ch.wmode = 1;
    else if (ch.wmode && ch.qw_n < c.wq_lo) ch.wmode = 0;
    only = ch.wmode ? 1u : (ch.q_n > ch.qw_n ? 0u : 1u);
  }
  // ---- column command ----
  bool col = false;
  uint32_t col_bank = 0;
  uint64_t oldest_age = ~0ull;
  if (c.dram_sched == 0) {  // FIFO: only the oldest request may issue (column and row commands)
    int o = P::argmin(qn, [&](int i) -> uint64_t {
      return (ch.q_valid[i] && (only == 2 || ch.q[i].write == only)) ? ch.q_age[i] : ~0ull;
    });
    oldest_age = o >= 0 ? ch.q_age[o] : ~0ull;
  }
  // no column command can issue before tCCD has elapsed: skip the scan
  if (t >= ch.t_ccd_ok) {
    int pick = P::argmin(qn, [&](int i) -> uint64_t {
      if (!ch.q_valid[i]) return ~0ull;
      if (c.dram_sched == 0 && ch.q_age[i] != oldest_age) return ~0ull;
      const DramReq& r = ch.q[i];
      if (only != 2 && r.write != only) return ~0ull;
      const DramBank& b = ch.bk[r.bank];
      if (!b.open || b.row != r.row || t < b.t_col_ok || t < ch.t_ccd_ok) return ~0ull;
      if (t < ch.t_ccdl_ok[dram_bkgrp(c, r.bank) & 7]) return ~0ull;
      if (r.write ? (t < ch.t_wr_ok) : (t < ch.t_rd_ok)) return ~0ull;
      return ch.q_age[i];
    });
    if (pick >= 0 && !(ch.q[pick].write == 0 && ch.ret_n >= (uint32_t)kDramRet)) {
      const DramReq r = ch.q[pick];
      DramBank& b = ch.bk[r.bank];
      if (trace_mem_on(c, TS_MEMORY_PARTITION_UNIT, ch.id))
        P::one([&] { trace_put(c, c.n_sm + ch.id, t, EV_DRAM_CMD, r.write ? 1 : 0, (uint64_t)r.bank << 32 | r.row); });
      if (r.write) {
        b.t_pre_ok = amax<uint64_t>(b.t_pre_ok, t + c.WL + burst + c.tWR);
        if (c.rw_turnaround) ch.t_rd_ok = amax<uint64_t>(ch.t_rd_ok, t + c.WL + burst + c.tCDLR);
        st.dram_wr++;
      } else {
        DramRet& o = ch.ret[(ch.ret_head + ch.ret_n) % kDramRet];
        o.line = r.line;
        o.sector = r.sector;
        o.sub = r.sub;
        o.ready = (t + c.CL + burst) * c.per_dram + (x.mall ? c.mall_miss_fs : 0);
        ch.ret_n++;
        b.t_pre_ok = amax<uint64_t>(b.t_pre_ok, t + c.tRTPL);
        uint64_t rtw = t + c.CL + burst + 2;
        if (c.rw_turnaround) ch.t_wr_ok = amax<uint64_t>(ch.t_wr_ok, rtw > c.WL ? rtw - c.WL : 0);
        st.dram_rd++;
      }
      ch.t_ccd_ok = t + amax<uint32_t>(c.tCCD, burst);
      ch.t_ccdl_ok[dram_bkgrp(c, r.bank) & 7] = t + amax<uint32_t>(c.tCCDL, burst);
      st.dram_busy_cycles += burst;
      ch.q_valid[pick] = 0;
      while (ch.q_hi && !ch.q_valid[ch.q_hi - 1]) --ch.q_hi;
      ch.q_n--;
      ch.qw_n -= r.write ? 1 : 0;
      if (r.sub != kSubNone) ch.sp[r.sub].n_l2dram--;
      col = true;
      col_bank = r.bank;
    }
  }
  // ---- row command (dual bus: in the same cycle) ----
  if (col && !c.dual_bus) return;
  // banks that had a queued row hit at the start of the cycle (only FR-FCFS
  // consults them): the column command above removed one row-hit request and
  // changed no bank's open row, so its bank is added back
  const uint64_t hitmask = c.dram_sched == 0 ? 0ull : (P::vor(qn, [&](int i) -> uint64_t {
    if (!ch.q_valid[i]) return 0;
    const DramReq& r = ch.q[i];
    if (only != 2 && r.write != only) return 0;  // requests of the idle queue do not hold rows open
    const DramBank& b = ch.bk[r.bank];
    return (b.open && b.row == r.row) ? (1ull << r.bank) : 0ull;
  }) | (col ? 1ull << col_bank : 0ull));
  int act = P::argmin(qn, [&](int i) -> uint64_t {
    if (!ch.q_valid[i]) return ~0ull;
    if (c.dram_sched == 0 && ch.q_age[i] != oldest_age) return ~0ull;
    const DramReq& r = ch.q[i];
    if (only != 2 && r.write != only) return ~0ull;
    const DramBank& b = ch.bk[r.bank];
    if (b.open) {
      // FR-FCFS: precharge a row only when no queued request still hits it
      // (FIFO serves strictly in order, so the oldest request's row wins)
      if (b.row == r.row || t < b.t_pre_ok) return ~0ull;
      if (c.dram_sched != 0 && (hitmask >> r.bank & 1ull)) return ~0ull;
      return ch.q_age[i];
    }
    if (t < b.t_act_ok || t < ch.t_rrd_ok) return ~0ull;
    return ch.q_age[i];
  });
  if (act >= 0) {
    const DramReq& r = ch.q[act];
    DramBank& b = ch.bk[r.bank];
    if (trace_mem_on(c, TS_MEMORY_PARTITION_UNIT, ch.id))
      P::one([&] {
        trace_put(c, c.n_sm + ch.id, t, EV_DRAM_CMD, b.open ? 3 : 2,
                  (uint64_t)r.bank << 32 | (b.open ? b.row : r.row));
      });
    if (b.open) {
      b.open = 0;
      b.t_act_ok = amax<uint64_t>(b.t_act_ok, t + c.tRP);
      st.dram_pre++;
    } else {
      b.open = 1;
      b.row = r.row;
      b.t_col_ok = t + c.tRCD;
      b.t_pre_ok = t + c.tRAS;
      b.t_act_ok = t + c.tRC;
      ch.t_rrd_ok = t + c.tRRD;
      st.dram_act++;
    }
  }
}

SIM_HDI bool sub_idle(const SubPart& sp) {
  return sp.inq_n == 0 && sp.ovf_n == 0 && sp.rop_n == 0 && sp.rep_n == 0 && sp.fill_n == 0 && sp.n_wait == 0 && sp.n_l2dram == 0;
}
SIM_HDI bool chan_idle(const ChanState& ch, const SimCfg& c) {
  if (ch.lat_n || ch.q_n || ch.ret_n || ch.mret_n) return false;
  for (uint32_t j = 0; j < c.n_sub_per_mem; ++j)
    if (!sub_idle(ch.sp[j])) return false;
  return true;
}

// advance the tick clocks of an idle channel to the first tick >= t1
SIM_HDI uint64_t next_tick(uint64_t t, uint64_t per, uint64_t t1) {
  if (t >= t1) return t;
  uint64_t k = (t1 - t + per - 1) / per;
  return t + k * per;
}

// Earliest time (fs) at which a tick of this channel can do more than add its
// per-tick statistics; `now` when something may happen right away.  A
// request that is ready but blocked (full queue, no credit) also counts as
// "now", so only pure waiting is skipped: requests riding the ROP delay
// queue, the L2->DRAM latency pipe or the DRAM data return, and arrivals not
// yet due.  Busy DRAM scheduler queues are never skipped (bank timing
// changes every cycle).  ~0 = nothing pending at all.
SIM_HDI uint64_t chan_next_event(const ChanState& ch, const SimCfg& c, uint64_t now) {
  if (ch.q_n) return now;
  uint64_t nx = ~0ull;
  if (ch.lat_n) nx = amin(nx, ch.lat[ch.lat_head].ready);
  if (ch.ret_n) nx = amin(nx, ch.ret[ch.ret_head].ready);
  if (ch.mret_n) nx = amin(nx, ch.mret[ch.mret_head].ready);
  for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
    const SubPart& sp = ch.sp[j];
    if (sp.rep_n || sp.ovf_n) return now;
    if (sp.fill_n) nx = amin(nx, sp.fill[sp.fill_head].ready);
    if (sp.rop_n) nx = amin(nx, sp.rop[sp.rop_head].t);
    if (sp.inq_n && sp.rop_n < (uint32_t)kRopQ && sp.rop_n < c.q_icnt_l2 + c.rop_latency)
      nx = amin(nx, sp.inq[sp.inq_head].t);
  }
  return nx > now ? nx : now;
}

// advance every clock domain of a quiet channel to its first tick >= target,
// adding exactly the statistics those ticks would have added (l2_cycle /
// dram_cycle with nothing ready)
SIM_HDI void chan_quiet_advance(ChanState& ch, const SimCfg& c, uint64_t target) {
  const uint64_t nd = next_tick(ch.t_dram, c.per_dram, target);
  const uint64_t kd = fdiv(nd - ch.t_dram, c.dv_dram);
  ch.sp[0].st.dram_cycles += kd;
  ch.sp[0].st.dram_q_occ += (uint64_t)ch.q_n * kd;
  ch.dcycle += kd;
  ch.t_dram = nd;
  const uint64_t nl = next_tick(ch.t_l2, c.per_l2, target);
  const uint64_t kl = fdiv(nl - ch.t_l2, c.dv_l2);
  for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
    ch.sp[j].st.l2_cycles += kl;
    ch.sp[j].st.rop_occ += (uint64_t)ch.sp[j].rop_n * kl;
  }
  ch.t_l2 = nl;
  ch.t_icnt = next_tick(ch.t_icnt, c.per_icnt, target);
}

// simulate all memory-side clock ticks in [.., x.win_end)
template <class P>
SIM_HDI void mem_window(ChanState& ch, const MemCtx& x) {
  const SimCfg& c = *x.cfg;
  const uint64_t t1 = x.win_end;
  if (chan_idle(ch, c)) {
    // nothing can happen until a new arrival (next epoch): skip the ticks
    uint64_t nd = next_tick(ch.t_dram, c.per_dram, t1);
    ch.sp[0].st.dram_cycles += fdiv(nd - ch.t_dram, c.dv_dram);
    ch.dcycle += fdiv(nd - ch.t_dram, c.dv_dram);
    ch.t_dram = nd;
    uint64_t nl = next_tick(ch.t_l2, c.per_l2, t1);
    for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) ch.sp[j].st.l2_cycles += fdiv(nl - ch.t_l2, c.dv_l2);
    ch.t_l2 = nl;
    ch.t_icnt = next_tick(ch.t_icnt, c.per_icnt, t1);
    return;
  }
  for (;;) {
    uint64_t tm = amin(ch.t_dram, amin(ch.t_l2, ch.t_icnt));
    if (tm >= t1) break;
    if (c.event_skip) {
      // fast-forward ticks in which provably nothing but statistics happens
      const uint64_t nx = chan_next_event(ch, c, tm);
      if (nx > tm) {
        chan_quiet_advance(ch, c, amin(nx, t1));
        continue;
      }
    }
    if (ch.t_dram == tm) {
      P::prof(21);
      dram_cycle<P>(ch, c, x, tm);
      ch.t_dram += c.per_dram;
    }
    if (ch.t_l2 == tm) {
      P::prof(22);
      for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) l2_cycle<P>(ch, ch.sp[j], c, j, tm);
      ch.t_l2 += c.per_l2;
    }
    if (ch.t_icnt == tm) {
      P::prof(23);
      for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) mem_icnt_cycle<P>(ch, ch.sp[j], c, x, j, tm);
      ch.t_icnt += c.per_icnt;
    }
    P::prof(24);
  }
}

// Gather one epoch of arrivals from the n_src source rows of an outbox cell
// array ([dst][src][cap], counts [dst][src]) and append them to `q` sorted by
// (time, source).  Keys are epoch-relative so they fit with the source id.
//
// Arrivals that do not fit in `q` are appended, in the same order, to the
// destination's backlog ring `ovf` (global memory) when one is given; the
// backlog is older than any new arrival and drains into `q` first on the next
// gathers.  This is the input buffering of the reference's interconnect
// (icnt input buffers, local_interconnect.cc:325-358) without a size limit of
// its own: the senders' outstanding-packet limit bounds it.  Without a
// backlog (SM side: replies <= outstanding requests <= queue size) nothing
// can overflow.
struct Backlog {
  Pkt* ring;          // nullptr = none
  uint32_t cap;
  uint32_t* head;
  uint32_t* n;
  uint64_t* drop;     // packets lost because the ring itself was full
};

template <class P>
SIM_HDI uint32_t gather_sorted(const Pkt* box, const uint32_t* cnt, uint32_t dst, uint32_t n_src,
                               uint32_t cap, uint64_t t0, Pkt* q, uint32_t qcap, uint32_t& qhead,
                               uint32_t& qn, uint64_t* skey, uint32_t* sref, uint32_t* srank,
                               uint32_t scap, const Backlog& bl = Backlog{nullptr, 0, nullptr, nullptr, nullptr}) {
  // 1. older backlog first (FIFO)
  if (bl.ring && *bl.n) {
    const uint32_t m = amin<uint32_t>(*bl.n, qcap - qn);
    const uint32_t h = *bl.head;
    P::each((int)m, [&](int i) { q[(qhead + qn + (uint32_t)i) % qcap] = bl.ring[(h + (uint32_t)i) % bl.cap]; });
    P::sync();
    qn += m;
    *bl.head = (h + m) % bl.cap;
    *bl.n -= m;
  }
  const uint32_t* row = cnt + (uint64_t)dst * n_src;
  // exclusive scan of the per-source counts -> slot of each packet
  const uint32_t total = P::scan((int)n_src, [&](int s) -> uint32_t { return row[s]; },
                                 [&](int s, uint32_t off) { srank[s] = off; });
  P::sync();
  if (total == 0) return 0;
  const Pkt* cell0 = box + (uint64_t)dst * n_src * cap;
  const uint32_t room = (bl.ring && *bl.n) ? 0u : qcap - qn;  // a non-empty backlog keeps order
  const uint32_t n = total < room ? total : room;
  // place the packet of rank r: queue slot or backlog tail
  auto place = [&](uint32_t r, const Pkt& p) {
    if (r < n) {
      q[(qhead + qn + r) % qcap] = p;
    } else if (bl.ring) {
      const uint32_t o = r - n;
      if (*bl.n + o < bl.cap) bl.ring[(*bl.head + *bl.n + o) % bl.cap] = p;
    }
  };
  if (total <= scap) {
    P::each((int)n_src, [&](int s) {
      uint32_t cnt_s = row[s], off = srank[s];
      for (uint32_t k = 0; k < cnt_s; ++k) {
        const Pkt& p = cell0[(uint64_t)s * cap + k];
        skey[off + k] = ((p.t - t0) << 16) | (uint64_t)s;
        sref[off + k] = ((uint32_t)s << 16) | k;
      }
    });
    P::sync();
    // rank sort (keys are unique: one packet per source per tick)
    P::each((int)total, [&](int i) {
      uint64_t k = skey[i];
      uint32_t r = 0;
      for (uint32_t j = 0; j < total; ++j) r += skey[j] < k;
      srank[i] = r;
    });
    P::sync();
    P::each((int)total, [&](int i) {
      const uint32_t s = sref[i] >> 16, k = sref[i] & 0xffff;
      place(srank[i], cell0[(uint64_t)s * cap + k]);
    });
    P::sync();
  } else {
    // more arrivals than sort scratch (many sources hitting one destination):
    // rank every packet against the time-ordered source rows directly
    P::each((int)n_src, [&](int s) {
      for (uint32_t k = 0; k < row[s]; ++k) {
        const Pkt& p = cell0[(uint64_t)s * cap + k];
        const uint64_t key = ((p.t - t0) << 16) | (uint64_t)s;
        uint32_t r = 0;
        for (uint32_t s2 = 0; s2 < n_src; ++s2)
          for (uint32_t k2 = 0; k2 < row[s2]; ++k2) {
            const uint64_t key2 = ((cell0[(uint64_t)s2 * cap + k2].t - t0) << 16) | (uint64_t)s2;
            if (key2 >= key) break;  // rows are time ordered
            ++r;
          }
        place(r, p);
      }
    });
    P::sync();
  }
  qn += n;
  if (bl.ring && total > n) {
    const uint32_t extra = total - n, fit = amin<uint32_t>(extra, bl.cap - *bl.n);
    *bl.n += fit;
    *bl.drop += extra - fit;
  }
  return n;
}

// bit d % 128 of a 128-bit destination mask (nullptr: every destination)
SIM_HDI bool dst_maybe(const uint64_t* m, uint32_t d) {
  return !m || ((m[(d >> 6) & 1u] >> (d & 63)) & 1ull);
}

template <class P>
SIM_HDI void mem_gather(ChanState& ch, const SimCfg& c, const MemCtx& x, const Pkt* box, const uint32_t* cnt,
                        uint32_t cap, uint64_t t0, const uint64_t* req_dst = nullptr) {
  for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
    SubPart& sp = ch.sp[j];
    uint32_t gsub = ch.id * c.n_sub_per_mem + j;
    // no request for this sub-partition last epoch and no backlog: nothing to move
    if (!dst_maybe(req_dst, gsub) && !(x.ovf && P::uni(sp.ovf_n))) continue;
    Backlog bl{x.ovf ? x.ovf + (uint64_t)gsub * x.ovf_cap : nullptr, x.ovf_cap, &sp.ovf_head, &sp.ovf_n,
               &sp.st.icnt_ovf_drop};
    gather_sorted<P>(box, cnt, gsub, c.n_sm, cap, t0, sp.inq, kMemInQ, sp.inq_head, sp.inq_n, ch.skey,
                     ch.sref, ch.srank, kMemInQ, bl);
  }
}

// publish this epoch's reply counts (every cell, zeros included) and reset
template <class P>
SIM_HDI void mem_publish(ChanState& ch, const SimCfg& c, uint32_t* outcnt, uint32_t cur, uint64_t* dm) {
  // destination SMs written this epoch (bit d % 128); the cells of parity
  // `cur` are rewritten only if they or the last write to them hold packets
  if (P::uni(ch.min_emit) != ~0ull)
    for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
      dm[0] |= P::vor((int)c.n_sm, [&](int d) -> uint64_t { return (ch.ocnt[j][d] && !(d & 64)) ? 1ull << (d & 63) : 0; });
      dm[1] |= P::vor((int)c.n_sm, [&](int d) -> uint64_t { return (ch.ocnt[j][d] && (d & 64)) ? 1ull << (d & 63) : 0; });
    }
  const uint32_t nzb = 1u << cur, nz = P::uni((uint32_t)ch.pub_nz);
  if ((dm[0] | dm[1]) || (nz & nzb)) {
    for (uint32_t j = 0; j < c.n_sub_per_mem; ++j) {
      uint32_t gsub = ch.id * c.n_sub_per_mem + j;
      P::each((int)c.n_sm, [&](int d) {
        outcnt[(uint64_t)d * c.n_subpart + gsub] = ch.ocnt[j][d];
        ch.ocnt[j][d] = 0;
      });
    }
    P::sync();
  }
  ch.pub_nz = (dm[0] | dm[1]) ? (nz | nzb) : (nz & ~nzb);
}

}  // namespace asim
