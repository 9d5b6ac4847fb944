// Cycle model of one SIMT core (SM / CU).  Single source for both engines.
//
// Stage order per cycle mirrors the reference's reverse-pipeline walk
// (shader_core_ctx::cycle, shader.cc:3629-3641: writeback -> execute ->
// read_operands -> issue -> decode/fetch) so an instruction advances at most
// one stage per cycle.  The data structures are re-designed for a 64-lane
// wavefront owning the SM: warps are lanes, the scheduler pick is a ballot +
// rotate + ffs (reference scheduler_unit::cycle, shader.cc:1249-1556 walks an
// STL vector), the scoreboard is a 256-bit mask per warp
// (scoreboard.cc:83-150 uses std::set), L1 ways are probed lane-parallel, and
// MSHR waiters live in a flat associative table instead of linked lists
// (mshr_table, gpu-cache.h:1019).
#pragma once
#include <stddef.h>
#if !defined(__HIP_DEVICE_COMPILE__)
#include <stdexcept>
#include <stdio.h>
#endif

#include "addrdec.h"

namespace asim {


// Warps read their instructions straight from the kernel's decoded trace
// (KernelDesc::insts, HBM on the GPU): w_next / w_head / w_end index it, with
// the kernel slot in the top bits (inst_at, types.h).

enum WarpFlags : uint8_t {
  WF_ACTIVE = 1,
  WF_EXITING = 2,    // EXIT issued / stream exhausted: no more fetch/issue
  WF_BARRIER = 4,    // waiting at a CTA barrier
  WF_MEMBAR = 8,     // waiting for outstanding stores
  WF_WAITCNT = 16,   // waiting for all outstanding memory (CDNA s_waitcnt)
  WF_IMISS = 32,     // instruction-cache miss pending (reference imiss_pending)
};

// hit / shared-memory completion ring entries
struct HitEnt {
  uint8_t warp;
  uint8_t slot;   // load slot, 0xff = store completion (inflight--)
  uint8_t kind;   // 0 = load access, 1 = store/shared-store done
  uint8_t pad;
};

struct WbEnt {
  uint8_t warp;
  uint8_t dst0;
  uint8_t dst1;
  uint8_t pad;
};

// ID_OC pipeline registers (one per scheduler per unit type, index
// sched * U_COUNT + unit == its idoc_mask bit) and operand collector units
// are kept as SoA columns: the instruction copies stay in memory, the small
// per-entry fields are single words that the GPU engine's register view holds
// one entry per lane (csrc/engine/sm_view.h).
//   idoc_meta: warp | load slot << 8 | age << 32
//   oc_info:   warp | sched << 8 | unit << 16 | load slot << 24 | lat << 32 | ii << 48
//   oc_banks:  bytes 0-4 bank of each pending operand read (0xff = none),
//              byte 5 reads left, byte 6 dst0, byte 7 dst1
constexpr int kIdOc = kMaxSched * U_COUNT;
SIM_HDI uint64_t idoc_pack(uint32_t warp, uint32_t slot, uint32_t age) {
  return (uint64_t)warp | (uint64_t)slot << 8 | (uint64_t)age << 32;
}

struct L1Line {
  uint64_t tag;      // line address
  uint32_t lru;      // last-use / insertion stamp
  uint8_t valid;     // sector mask (readable sectors)
  uint8_t dirty;     // sector mask (write-back data not yet written below)
  uint8_t pad[2];
};

struct L1Mshr {
  uint64_t line;
  uint8_t requested;  // sectors requested from L2
  uint8_t valid;      // entry in use
  uint8_t merges;
  uint8_t pad;
  uint32_t t_issue;   // core cycle (low 32 bits) the miss was sent: memory latency stats
};

struct L1Pend {  // a load access waiting for sectors of a line
  uint64_t line;
  uint8_t need;   // sectors
  uint8_t warp;
  uint8_t slot;
  uint8_t valid;
  uint32_t pad;
};

struct LdstState {
  TInst inst;
  uint8_t busy;
  uint8_t warp;
  uint8_t slot;
  uint8_t next;       // next access index
  uint32_t start;     // cycle the instruction entered the unit (low 32 bits)
  uint32_t port_free; // -sim_l1_port_bytes: first cycle the L1 data path is free again (low 32 bits)
  uint32_t pad;
};

// statistics counters of one SM (reduced on the host)
enum L1StatType : uint8_t { L1T_GLOBAL_R = 0, L1T_GLOBAL_W, L1T_LOCAL_R, L1T_LOCAL_W, L1T_ATOMIC, L1T_COUNT };
enum L1StatOut : uint8_t { L1O_HIT = 0, L1O_MISS, L1O_MSHR_HIT, L1O_RES_FAIL, L1O_BYPASS, L1O_COUNT };
struct SMStats {
  uint64_t thread_insn;        // gpu_sim_insn contribution (active-thread count)
  uint64_t warp_insn;
  uint64_t cls_insn[OC_COUNT];
  uint64_t active_cycles;      // cycles with at least one live warp
  uint64_t busy_cycles;        // cycles with at least one instruction issued
  uint64_t issue_stall_idle;   // scheduler cycles with no ready warp
  uint64_t sb_stall;           // warps blocked by scoreboard (sampled per cycle)
  uint64_t pipe_stall;
  uint64_t l1[L1T_COUNT][L1O_COUNT];
  uint64_t shmem_acc;
  uint64_t shmem_conflict_cycles;
  uint64_t pkts_out;
  uint64_t pkts_in;
  uint64_t bytes_out;
  uint64_t bytes_in;
  uint64_t rf_reads;
  uint64_t rf_writes;
  uint64_t oc_bank_conflicts;
  uint64_t ctas_done;
  uint64_t warps_done;
  uint64_t occupancy_acc;      // sum over cycles of live warps
  uint64_t mem_insn;
  uint64_t power_acc[16];      // power-model counters (PwrCounter)
  // L1 miss round-trip latency (MSHR allocation -> last sector filled), the
  // reference's mem_latency_stat (mem_latency_stat.h:37, -gpgpu_memlatency_stat)
  uint64_t mf_lat_sum, mf_lat_n, mf_lat_max;
  uint64_t mf_lat_hist[16];    // log2 buckets: [2^i, 2^(i+1)) cycles
  uint64_t il1[4];             // instruction cache: hit, miss, mshr (pending) hit, reservation fail
  uint64_t il1_prefetch;       // code lines requested by the sequential prefetcher
  uint64_t cl1[4];             // constant / scalar data cache: hit, miss, mshr (pending) hit, reservation fail
  uint64_t dual_issued;        // second instructions issued in the same cycle by one warp
  uint64_t l1_wb;              // dirty L1 lines written back on eviction
  uint64_t l1_wb_lost;         // write-backs dropped with the injection queue full (must stay 0)
  uint64_t icnt_reply_conflicts;     // reply net: ready inputs not granted by this SM's ejection port
  uint64_t icnt_reply_queue_cycles;  // reply net: icnt cycles granted replies waited at the port
  uint64_t sq_insn[8];               // issued wave instructions by the CDNA SQ counter classes (SqClass)
  // reference shader_core_stats::shader_cycle_distro (shader.cc:724-730,
  // 1045, 1547-1555), per scheduler and cycle: [0] W0_Idle (no warp with a
  // valid instruction), [1] W0_Scoreboard (valid instructions all wait on the
  // scoreboard), [2] Stall (ready, but the pipeline did not take it), and
  // [2 + k] one instruction issued with k active threads (k = 1..64)
  uint64_t issue_distro[3 + kMaxWarpLanes];
  uint64_t single_issue[kMaxSched];  // scheduler cycles that issued one instruction
  uint64_t dual_issue[kMaxSched];    // ... two
  // vector-L1 tag lookups at 64 B granularity (the 64 B halves of each
  // coalesced 128 B line access): what TCP_TOTAL_CACHE_ACCESSES counts
  uint64_t l1_lookups64;
  // cycles a ready packet waited for room in the router's injection queue
  // (-icnt_link_contention 2 back-pressure)
  uint64_t icnt_inj_stall;
};
enum IL1Out : uint8_t { IL1_HIT = 0, IL1_MISS, IL1_MSHR_HIT, IL1_RES_FAIL };
// Instruction classes of the CDNA sequencer's counters (rocprofv3
// SQ_INSTS_VALU / _SALU / _SMEM / _VMEM_RD / _VMEM_WR / _LDS / _BRANCH; VALU
// includes MFMA), derived from the decoded class and memory space; OTHER =
// s_waitcnt / s_nop / s_barrier / s_endpgm and friends, which no SQ_INSTS_*
// class counts (isatrace/verify.py classify() is the mnemonic-level twin)
enum SqClass : uint8_t { SQ_VALU = 0, SQ_SALU, SQ_SMEM, SQ_VMEM_RD, SQ_VMEM_WR, SQ_LDS, SQ_BRANCH, SQ_OTHER };
SIM_HDI uint32_t sq_class(const TInst& in) {
  switch (in.cls) {
    case OC_LOAD: return in.space == S_SHARED ? SQ_LDS : in.space == S_CONST ? SQ_SMEM : SQ_VMEM_RD;
    case OC_STORE: return in.space == S_SHARED ? SQ_LDS : in.space == S_CONST ? SQ_SMEM : SQ_VMEM_WR;
    case OC_BRANCH: return SQ_BRANCH;
    case OC_SPEC8: return SQ_SALU;  // CDNA traces put the scalar ALU on specialized unit 8
    case OC_BARRIER:
    case OC_MEMBAR:
    case OC_EXIT:
    case OC_NOP: return SQ_OTHER;
    default: return in.space == S_CONST ? SQ_SMEM : SQ_VALU;  // s_memtime is an SMEM op
  }
}
// SMStats::power_acc slots: constant-cache operands, then the active lanes
// charged at issue per execution-unit kind (slot = the instruction's power
// kind, TInst::flags >> 4; reference incexecstat, shader.cc:3226-3290)
enum PwrCounter : uint8_t {
  PWR_CONST_OPERAND = 0,
  PWR_INT = 1, PWR_INT_MUL, PWR_FP, PWR_FP_MUL, PWR_DP, PWR_DP_MUL, PWR_SQRT, PWR_LG, PWR_SIN, PWR_EXP, PWR_TENSOR,
  PWR_TEX, PWR_SALU, PWR_KINDS
};
static_assert(PWR_KINDS <= 16, "power kinds live in the upper nibble of TInst::flags");


// Complete state of one SM.  On the GPU it lives in LDS for the duration of
// a launch (copied in/out of HBM), on the CPU it is a plain struct.
struct alignas(16) SMState {
  uint32_t id;
  uint16_t l1_sets, l1_assoc; // L1 geometry of the kernel that last found the SM empty (adaptive carve-out)
  uint64_t cycle;             // next core cycle to simulate
  uint64_t last_progress;     // last cycle an instruction completed (deadlock)
  uint64_t epoch_end;         // current epoch end cycle (exclusive)
  uint64_t out_port_free;     // cycle the injection port frees
  // -icnt_link_contention 2 injection back-pressure (icnt_router.h
  // rt_inj_allow0): the epoch's start (fs), its flit allowance at that start
  // and the flits injected since (times the SMs sharing the node)
  uint64_t inj_t0_fs;
  int64_t inj_allow0;
  uint64_t inj_used;
  uint32_t age_ctr;
  uint16_t arb_next, arb_cnt;  // reply-network output-port arbiter (xbar_pick)
  // ---- warps (SoA) ----
  uint32_t w_next[kMaxWarps];   // next trace index to fetch into ibuf
  uint32_t w_end[kMaxWarps];    // end of stream
  uint32_t w_head[kMaxWarps];   // next trace index to issue
  uint32_t w_age[kMaxWarps];    // dynamic warp id (oldest first)
  uint8_t w_flags[kMaxWarps];
  uint8_t w_ibuf[kMaxWarps];    // decoded instructions available
  uint8_t w_cta[kMaxWarps];
  uint8_t w_inflight[kMaxWarps];
  uint16_t w_stores[kMaxWarps];  // outstanding store acks
  uint16_t w_loads[kMaxWarps];   // outstanding load slots in use
  uint16_t w_wait[kMaxWarps];    // counts of the pending s_waitcnt: vm | lgkm << 8 (0xff: not waited for)
  uint64_t w_sb[kMaxWarps][4];   // scoreboard: pending destination registers
  uint64_t w_issue_ok[kMaxWarps];  // first cycle the warp may issue again (-gpgpu_warp_issue_interval)
  uint8_t w_slot_used[kMaxWarps];  // bitmask of used load slots
  uint8_t w_slot_lds[kMaxWarps];   // load slots holding an LDS load (lgkmcnt, not vmcnt)
  uint8_t w_lds_st[kMaxWarps];     // LDS stores in flight (lgkmcnt)
  uint8_t w_pad[kMaxWarps];
  uint16_t w_slot_pend[kMaxWarps][kLoadSlots];
  uint8_t w_slot_dst[kMaxWarps][kLoadSlots][2];
  // ---- CTAs ----
  uint32_t cta_id[kMaxCta];
  uint8_t cta_valid[kMaxCta];
  uint8_t cta_live[kMaxCta];     // warps not yet completed
  uint8_t cta_bar[kMaxCta];      // warps arrived at barrier
  uint8_t cta_nexit[kMaxCta];    // warps exited (excluded from barrier count)
  uint8_t cta_ks[kMaxCta];       // kernel slot of the CTA
  uint8_t cta_wbase[kMaxCta];    // first warp of the CTA (its warps are contiguous)
  uint8_t cta_nw[kMaxCta];       // warps of the CTA
  uint8_t n_cta_k[kMaxConc];     // CTAs resident per kernel slot
  uint64_t cta_wmask;            // warps owned by resident CTAs
  uint32_t used_thr, used_regs, used_shmem;  // resources held by resident CTAs
  uint32_t n_cta_active;
  uint32_t n_warps_live;         // warps with WF_ACTIVE (occupancy statistic)
  uint64_t live_mask;            // bit w: warp w has WF_ACTIVE
  uint32_t n_wait_flags;         // warps parked in WF_MEMBAR / WF_WAITCNT
  // ---- front end ----
  uint32_t fetch_rr;
  uint32_t sched_last[kMaxSched];
  // ---- pipeline registers / operand collectors / FUs ----
  TInst idoc_inst[kIdOc];
  uint64_t idoc_meta[kIdOc];
  TInst oc_inst[kMaxOC];
  uint64_t oc_info[kMaxOC];
  uint64_t oc_banks[kMaxOC];
  uint32_t oc_age[kMaxOC];
  uint32_t fu_next[U_COUNT * kMaxSched];  // [unit * kMaxSched + phys]: cycle (low 32) the unit can accept again
  // ---- LD/ST + L1 ----
  LdstState ldst;
  TAcc ldst_acc[kMaxAccess];     // access records of the instruction in the LD/ST unit (loaded at dispatch)
  uint32_t n_pend;
  uint64_t w_iline[kMaxWarps];  // code line a WF_IMISS warp waits for
  uint64_t idoc_mask;     // bit sched*U_COUNT+unit: ID_OC register occupied
  uint32_t oc_mask;       // occupied operand collectors
  uint32_t oc_read_mask;  // collectors still reading operands
  uint32_t l1_stamp;
  // occupancy bitmaps of the time-indexed rings (bit = slot holds entries):
  // the next completion time is a find-first-set instead of a ring scan
  uint64_t wb_occ[kWbRing / 64];
  uint64_t hit_occ[kHitRing / 64];
  uint64_t skipped_cycles;  // quiet cycles fast-forwarded inside epochs (diagnostic)
  uint64_t min_emit;        // earliest arrival time (fs) of the packets injected this epoch
  // ---- interconnect endpoints ----
  uint32_t outq_head, outq_n;
  uint32_t outstanding;     // packets awaiting a reply
  uint32_t pub_nz;          // bit p: the request cells of mailbox parity p were last written with packets
  uint32_t ocnt[kMaxSubTot]; // packets put into each destination's outbox cell this epoch
  uint32_t inq_head, inq_n;
  // reply path: cluster ejection buffer -> LD/ST response FIFO (sm_receive)
  Pkt rsp_cl[kEjectQ];
  Pkt rsp_ld[kLdstRespQ];
  uint32_t cl_head, cl_n, ld_head, ld_n;
  // replicated kernel dispatch state (identical in every SM): per slot, the
  // uid the SM initialised it for and the next CTA to hand out
  uint32_t k_uid[kMaxConc];
  uint32_t next_cta[kMaxConc];
  // -sim_xcd: CTAs go round-robin over the XCDs (CTA i to an SM of XCD
  // i % n_xcd, the hardware's workgroup dispatch); per XCD the CTAs of its
  // residue handed out so far (next_cta is then their sum)
  uint32_t next_ctax[kMaxConc][kMaxXcd];
  SMStats st;
  // ---- the geometry-sized arrays (SMTail: everything from wb_cnt on).  The
  // GPU engine's split-state build keeps the fields above in LDS and these
  // in the unit's HBM image (csrc/engine/sm_split.h SmSplit) ----
  alignas(16) uint8_t wb_cnt[kWbRing];
  // decoded instructions [w_head, w_next] of each warp (slot = index & (kWin-1)):
  // the fetched-not-issued ones plus the next fetch's target (its PC feeds the
  // instruction cache).  Filled from the trace at fetch / CTA launch (LDS DMA
  // in the LDS-state build; the split build reads them from the unit's HBM
  // image, an L2-resident line per warp, to keep a block's LDS at ~19 KB)
  TInst w_win[kMaxWarps][kWin];
  Pkt outq[kOutQ];  // interconnect injection queue (outq_head / outq_n above)
  Pkt inq[kInQ];    // arrived packets not yet ejected (inq_head / inq_n above)
  uint64_t skey[kInQ];  // gather scratch
  uint32_t sref[kInQ];
  uint32_t srank[kInQ > kMaxSubTot ? kInQ : kMaxSubTot];
  WbEnt wb[kWbRing][kWbSlot];
  uint8_t hit_cnt[kHitRing];
  HitEnt hit[kHitRing][kHitSlot];
  L1Line l1[kMaxL1Lines];
  L1Mshr mshr[kMaxL1Mshr];
  L1Pend pend[kMaxPend];
  L1Line il1[kMaxIL1Lines];     // instruction cache tags (non-sectored: valid = 0xf)
  L1Mshr imshr[kMaxIL1Mshr];
  L1Line cl1[kMaxCL1Lines];     // constant / scalar data cache tags (valid = 1: non-sectored)
  L1Mshr cmshr[kMaxCL1Mshr];
  // statistics by word index (SK below); the GPU engine's register view keeps
  // the counters in lanes during the cycle loop (csrc/engine/sm_view.h)
  SIM_HDI void sadd(uint32_t k, uint64_t d) { reinterpret_cast<uint64_t*>(&st)[k] += d; }
  SIM_HDI uint64_t sget(uint32_t k) const { return reinterpret_cast<const uint64_t*>(&st)[k]; }
  SIM_HDI void sset(uint32_t k, uint64_t v) { reinterpret_cast<uint64_t*>(&st)[k] = v; }
  // a counter at a run-time index k in [LO, HI) (one counter array, e.g. the
  // instruction class histogram): the GPU engine's register view touches
  // only the register words of that range (sm_view.h)
  template <uint32_t LO, uint32_t HI>
  SIM_HDI void sadd_r(uint32_t k, uint64_t d) { sadd(k, d); }
};
#define SK(f) ((uint32_t)(offsetof(::asim::SMStats, f) / 8))
// counter array `f` of n words, element i (run time)
#define SADD_IN(s, f, n, i, d) (s).template sadd_r<SK(f), SK(f) + (n)>(SK(f) + (uint32_t)(i), (d))
constexpr int kStatWords = (int)(sizeof(SMStats) / 8);
static_assert(kStatWords <= 256, "SM statistics: up to four 64-lane register words on the GPU engine");
template <class S>
SIM_HDI uint64_t* s_scratch_key(S& s) { return s.skey; }
template <class S>
SIM_HDI uint32_t* s_scratch_ref(S& s) { return s.sref; }
template <class S>
SIM_HDI uint32_t* s_scratch_rank(S& s) { return s.srank; }

// ---------------------------------------------------------------------------
// context passed to every SM step
struct SmCtx {
  const SimCfg* cfg;
  const KernelTab* kt;   // running kernels (instructions, access tables, CTA streams)
  Pkt* outbox;           // this epoch's outbox base: [dst][src][cap]
  uint32_t* outcnt;      // [dst][src]
  uint32_t out_cap;      // per (dst,src) capacity (>= epoch length)
  uint32_t n_src_sm;     // number of SMs (row stride)
  const uint64_t* rt_st = nullptr;  // -icnt_link_contention 2: the router model's state (injection back-pressure)
};

SIM_HDI uint32_t wb_width(const SimCfg& c) { return c.ex_wb_width < (uint32_t)kWbSlot ? c.ex_wb_width : (uint32_t)kWbSlot; }

SIM_HDI bool sb_test(const uint64_t* sb, uint8_t r) { return r && ((sb[r >> 6] >> (r & 63)) & 1ull); }
SIM_HDI void sb_set(uint64_t* sb, uint8_t r) {
  if (r) sb[r >> 6] |= 1ull << (r & 63);
}
SIM_HDI void sb_clr(uint64_t* sb, uint8_t r) {
  if (r) sb[r >> 6] &= ~(1ull << (r & 63));
}
// scoreboard by (warp, register): the GPU engine's register view overloads
// these for its per-lane scoreboard words (csrc/engine/sm_view.h)
template <size_t N>
SIM_HDI bool sbt(const uint64_t (&sb)[N][4], uint32_t w, uint8_t r) { return sb_test(sb[w], r); }
template <size_t N>
SIM_HDI void sbs(uint64_t (&sb)[N][4], uint32_t w, uint8_t r) { sb_set(sb[w], r); }
template <size_t N>
SIM_HDI void sbc(uint64_t (&sb)[N][4], uint32_t w, uint8_t r) { sb_clr(sb[w], r); }
template <size_t N>
SIM_HDI void sbz(uint64_t (&sb)[N][4], uint32_t w) { sb[w][0] = sb[w][1] = sb[w][2] = sb[w][3] = 0; }

// ---------------------------------------------------------------------------
// reset an SM for a new kernel (state persists across kernels otherwise:
// L1 may be flushed by -gpgpu_flush_l1_cache)
template <class P, class S>
SIM_HDI void sm_reset(S& s, uint32_t id) {
  // caller zero-fills the struct; set identity
  s.id = id;
}

// L1 geometry in use (adaptive per kernel: set when a CTA launches into an
// empty SM, shader_core_ctx::issue_block2core's cache reconfiguration)
template <class S>
SIM_HDI CacheGeom l1_geom(const SimCfg& c, const S& s) {
  CacheGeom g = c.l1;
  const uint32_t sets = s.l1_sets;
  if (sets) {
    g.nsets = sets;
    g.assoc = s.l1_assoc;
  }
  return g;
}

// ---------------------------------------------------------------------------
// injection: enqueue a packet towards the interconnect
template <class S>
SIM_HDI bool sm_can_send(const S& s, const SimCfg& c) {
  return s.outq_n < c.icnt_in_pkts && s.outstanding + s.outq_n < c.icnt_out_limit;
}
template <class S>
SIM_HDI bool sm_can_send_n(const S& s, const SimCfg& c, uint32_t n) {
  return s.outq_n + n <= c.icnt_in_pkts && s.outstanding + s.outq_n + n <= c.icnt_out_limit;
}
// write-back packets of evicted dirty L1 sectors carry this tag: their
// acknowledgement retires no warp store
constexpr uint32_t kTagL1Writeback = 0x20000000u;
template <class S>
SIM_HDI void sm_send(S& s, const SimCfg& c, uint8_t type, uint64_t line, uint8_t sectors,
                     uint16_t bytes, uint32_t tag) {
  AddrTlx t = addr_decode(c, line);
  Pkt& p = s.outq[(s.outq_head + s.outq_n) % kOutQ];
  p.addr = line;
  p.t = 0;
  p.tag = tag;
  p.src = (uint16_t)s.id;
  p.dst = (uint16_t)l2_slice_of(c, s.id, t.sub);
  p.type = type;
  p.sectors = sectors;
  p.size = (type == P_WR) ? (uint16_t)(8 + bytes) : (uint16_t)8;
  p.aux = 0;
  s.outq_n++;
}

// -sim_l1_write_request_bytes 64: the L1 sends a store as one request per
// 64 B half line it touches (gfx950's TCP -> TCC writes are at most 64 B:
// TCC_WRITE counts two requests for a 128 B store); 128 keeps one per line.
// Returns the number of packets (each is acknowledged).
template <class S>
SIM_HDI uint32_t wr_packets(const SimCfg& c, uint8_t sectors) {
  if (c.l1_wr_req_bytes != 64) return 1u;
  return ((sectors & 3u) && (sectors & 12u)) ? 2u : 1u;
}
template <class S>
SIM_HDI uint32_t sm_send_write(S& s, const SimCfg& c, uint64_t line, uint8_t sectors, uint16_t bytes, uint32_t tag) {
  if (wr_packets<S>(c, sectors) == 1) {
    sm_send(s, c, P_WR, line, sectors, bytes, tag);
    return 1;
  }
  const uint8_t lo = sectors & 3u, hi = sectors & 12u;
  const uint32_t n = (uint32_t)popc64(sectors);
  const uint16_t blo = (uint16_t)((uint32_t)bytes * (uint32_t)popc64(lo) / n);
  sm_send(s, c, P_WR, line, lo, blo, tag);
  sm_send(s, c, P_WR, line, hi, (uint16_t)(bytes - blo), tag);
  return 2;
}

// HasBuffer of the router model (icnt_router.h rt_inj_allow0): `nfl` more
// flits fit the node's injection queue at core cycle `now` of the epoch
SIM_HDI bool rt_inj_ok(const SimCfg& c, uint64_t t0_fs, int64_t allow0, uint64_t used, uint32_t nfl, uint64_t now_fs) {
  const uint64_t k = now_fs > t0_fs ? fdiv(now_fs - t0_fs, c.dv_icnt) : 0;
  return (int64_t)(used + nfl) <= allow0 + (int64_t)(k < (1ull << 40) ? k : (1ull << 40));
}

// move the head packet into the outbox once the injection port is free.  A
// multi-flit packet may finish serialising after the epoch ends (port_free
// carries over); its arrival time is still beyond the lookahead, so the
// epoch length does not gate injection (it did: with epochs shorter than a
// packet's flit count nothing could ever be sent)
template <class P, class S>
SIM_HDI void sm_inject(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  if (P::uni(s.outq_n) == 0) return;
  if (now < P::uni(s.out_port_free)) return;
  Pkt p = P::uni(s.outq[P::uni(s.outq_head)]);
  uint32_t nflits = (p.size + c.flit_size - 1) / c.flit_size;
  uint64_t done = now + nflits - 1;
  uint32_t dst = p.dst;
  uint32_t slot = dst * x.n_src_sm + s.id;
  uint32_t n = P::uni(s.ocnt[dst]);
  if (n >= x.out_cap) return;  // outbox cell full (cannot happen with cap >= epoch)
  const uint32_t cpc = c.cores_per_cluster ? c.cores_per_cluster : 1;
  if (c.link_contention == 2 &&
      !rt_inj_ok(c, P::uni(s.inj_t0_fs), P::uni(s.inj_allow0), P::uni(s.inj_used), nflits * cpc, core_fs(c, now))) {
    s.sadd(SK(icnt_inj_stall), 1);  // the node's injection queue is full
    return;
  }
  if (c.link_contention == 2) s.inj_used = s.inj_used + (uint64_t)nflits * cpc;
  s.ocnt[dst] = n + 1;
  p.t = core_fs(c, done) + icnt_pkt_lat_fs(c, s.id, dst);
  s.min_emit = amin(s.min_emit, p.t);
  if (trace_sm_on(c, TS_INTERCONNECT, s.id)) P::one([&] { trace_put(c, s.id, now, EV_PKT_SEND, (uint16_t)dst, p.addr); });
  P::one([&] {
    x.outbox[(uint64_t)slot * x.out_cap + n] = p;
    x.outcnt[slot] = n + 1;
  });
  s.outq_head = (s.outq_head + 1) % kOutQ;
  s.outq_n--;
  s.out_port_free = now + nflits;
  s.outstanding++;
  s.sadd(SK(pkts_out), 1);
  s.sadd(SK(bytes_out), p.size);
}

// ---------------------------------------------------------------------------
// writeback of ALU results due this cycle
template <class P, class S>
SIM_HDI void sm_writeback(S& s, const SimCfg& c, uint64_t now) {
  uint32_t slot = (uint32_t)(now % kWbRing);
  // the occupancy bitmap (registers on the GPU) says whether the slot holds
  // entries: an empty slot costs no ring access
  if (!((P::uni((uint64_t)s.wb_occ[slot >> 6]) >> (slot & 63)) & 1ull)) return;
  uint32_t n = P::uni(s.wb_cnt[slot]);
  for (uint32_t i = 0; i < n; ++i) {
    WbEnt e = P::uni(s.wb[slot][i]);
    if (trace_sm_on(c, TS_SCOREBOARD, s.id))
      P::one([&] {
        if (e.dst0) trace_put(c, s.id, now, EV_SB_RELEASE, e.warp, e.dst0 - 1u);
        if (e.dst1) trace_put(c, s.id, now, EV_SB_RELEASE, e.warp, e.dst1 - 1u);
      });
    sbc(s.w_sb, e.warp, e.dst0);
    sbc(s.w_sb, e.warp, e.dst1);
    s.w_inflight[e.warp]--;
    s.sadd(SK(rf_writes), (e.dst0 != 0) + (e.dst1 != 0));
  }
  if (n) s.last_progress = now;
  s.wb_cnt[slot] = 0;
  s.wb_occ[slot >> 6] &= ~(1ull << (slot & 63));
}

template <class S>
SIM_HDI void sm_load_slot_done(S& s, uint32_t w, uint32_t slot, uint64_t now) {
  sbc(s.w_sb, w, s.w_slot_dst[w][slot][0]);
  sbc(s.w_sb, w, s.w_slot_dst[w][slot][1]);
  s.sadd(SK(rf_writes), (s.w_slot_dst[w][slot][0] != 0) + (s.w_slot_dst[w][slot][1] != 0));
  s.w_slot_used[w] &= (uint8_t)~(1u << slot);
  s.w_slot_lds[w] &= (uint8_t)~(1u << slot);
  s.w_loads[w]--;
  s.w_inflight[w]--;
  s.last_progress = now;
}

// CDNA s_waitcnt: the wave may go on once at most vm vector-memory operations
// (global/local loads and store acknowledgements) and at most lgkm LDS
// operations are outstanding.  The hardware counters retire in issue order;
// here completions may come back out of order, so a younger fast access can
// release a count-based wait early.
template <class S>
SIM_HDI bool waitcnt_met(S& s, uint32_t w) {
  const uint32_t wt = s.w_wait[w];
  const uint32_t lds_ld = (uint32_t)__builtin_popcount((uint32_t)s.w_slot_lds[w]);
  const uint32_t vm = (uint32_t)s.w_loads[w] - lds_ld + (uint32_t)s.w_stores[w];
  const uint32_t lgkm = lds_ld + (uint32_t)s.w_lds_st[w];
  return vm <= (wt & 0xffu) && lgkm <= (wt >> 8);
}

// L1-hit / shared-memory completions due this cycle
template <class P, class S>
SIM_HDI void sm_hit_complete(S& s, uint64_t now) {
  uint32_t slot = (uint32_t)(now % kHitRing);
  if (!((P::uni((uint64_t)s.hit_occ[slot >> 6]) >> (slot & 63)) & 1ull)) return;  // empty slot
  uint32_t n = P::uni(s.hit_cnt[slot]);
  for (uint32_t i = 0; i < n; ++i) {
    HitEnt e = P::uni(s.hit[slot][i]);
    if (e.kind == 0) {
      if (--s.w_slot_pend[e.warp][e.slot] == 0) sm_load_slot_done(s, e.warp, e.slot, now);
    } else {
      s.w_inflight[e.warp]--;
      s.w_lds_st[e.warp]--;
      s.last_progress = now;
    }
  }
  s.hit_cnt[slot] = 0;
  s.hit_occ[slot >> 6] &= ~(1ull << (slot & 63));
}

template <class S>
SIM_HDI bool hit_push(S& s, uint64_t when, uint8_t warp, uint8_t slot, uint8_t kind) {
  uint32_t r = (uint32_t)(when % kHitRing);
  if (s.hit_cnt[r] >= kHitSlot) return false;
  s.hit_occ[r >> 6] |= 1ull << (r & 63);
  HitEnt& e = s.hit[r][s.hit_cnt[r]++];
  e.warp = warp;
  e.slot = slot;
  e.kind = kind;
  e.pad = 0;
  return true;
}

// a load access whose data came back from below the L1 (fill or bypassing
// reply): completes now, or -sim_l1_miss_return_latency cycles later through
// the completion ring (the first ring slot at or after that cycle with room)
template <class S>
SIM_HDI void sm_miss_access_done(S& s, const SimCfg& c, uint32_t w, uint32_t sl, uint64_t now) {
  if (c.l1_miss_ret) {
    for (uint32_t d = 0; d < 16; ++d)
      if (hit_push(s, now + c.l1_miss_ret + d, (uint8_t)w, (uint8_t)sl, 0)) return;
  }
  if (--s.w_slot_pend[w][sl] == 0) sm_load_slot_done(s, w, sl, now);
}

// ---------------------------------------------------------------------------
// L1 data cache (sectored, lane-parallel probe over the ways of a set)
template <class P, class S>
SIM_HDI int l1_find(const S& s, const CacheGeom& g, uint32_t set, uint64_t line) {
  const L1Line* base = &s.l1[set * g.assoc];
  const int assoc = (int)g.assoc;
  if (assoc <= 64) {
    uint64_t m = P::ballot(assoc, [&](int w) { return base[w].valid && base[w].tag == line; });
    return m ? ffs64(m) : -1;
  }
  for (int b = 0; b < assoc; b += 64) {
    int n = amin(64, assoc - b);
    uint64_t m = P::ballot(n, [&](int w) { return base[b + w].valid && base[b + w].tag == line; });
    if (m) return b + ffs64(m);
  }
  return -1;
}

template <class P, class S>
SIM_HDI int l1_victim(const S& s, const CacheGeom& g, uint32_t set) {
  const L1Line* base = &s.l1[set * g.assoc];
  // invalid way first (lowest index), else smallest stamp (LRU or FIFO)
  int v = P::argmin((int)g.assoc, [&](int w) -> uint64_t {
    return base[w].valid ? (1ull << 40) | base[w].lru : (uint64_t)w;
  });
  return v;
}

// evict L1 line `idx`: dirty (write-back) sectors go below (reference
// data_cache eviction write-back, gpu-cache.cc:1372-1386).  With the
// injection queue full the write-back is counted as lost instead.
template <class P, class S>
SIM_HDI void l1_evict(S& s, const SimCfg& c, uint32_t idx) {
  L1Line& V = s.l1[idx];
  const uint8_t d = P::uni(V.dirty);
  if (V.valid | d) {
    if (d) {
      if (s.outq_n < (uint32_t)kOutQ) {
        sm_send(s, c, P_WR, P::uni(V.tag), d, (uint16_t)(32 * popc64(d)), kTagL1Writeback);
        s.sadd(SK(l1_wb), 1);
      } else {
        s.sadd(SK(l1_wb_lost), 1);
      }
    }
  }
  V.valid = 0;
  V.dirty = 0;
}

// fill sectors of a line into L1 (allocate-on-fill) and wake waiters
template <class P, class S>
SIM_HDI void l1_fill(S& s, const SmCtx& x, uint64_t line, uint8_t sectors, uint64_t now) {
  const SimCfg& c = *x.cfg;
  const CacheGeom g = l1_geom(c, s);
  if (!g.disabled) {
    uint32_t set = cache_set_index(g, line);
    int w = l1_find<P>(s, g, set, line);
    if (w < 0) {
      w = l1_victim<P>(s, g, set);
      l1_evict<P>(s, c, set * g.assoc + w);
      L1Line& L = s.l1[set * g.assoc + w];
      L.tag = line;
      L.valid = 0;
      L.dirty = 0;
      L.lru = ++s.l1_stamp;
    }
    L1Line& L = s.l1[set * g.assoc + w];
    L.valid |= sectors;
    if (g.repl == REPL_LRU) L.lru = ++s.l1_stamp;
  }
  // mshr bookkeeping
  int mi = P::find_first((int)c.l1.mshr_entries, [&](int i) -> bool { return s.mshr[i].valid && s.mshr[i].line == line; });
  if (mi >= 0) {
    s.mshr[mi].requested &= (uint8_t)~sectors;
    if (s.mshr[mi].requested == 0) {
      s.mshr[mi].valid = 0;
      const uint32_t lat = (uint32_t)now - s.mshr[mi].t_issue;
      s.sadd(SK(mf_lat_sum), lat);
      s.sadd(SK(mf_lat_n), 1);
      if (lat > s.sget(SK(mf_lat_max))) s.sset(SK(mf_lat_max), lat);
      SADD_IN(s, mf_lat_hist, 16, lat ? amin<int>(15, 31 - __builtin_clz(lat)) : 0, 1);
    }
  }
  // wake waiters whose sectors are now all present (lane-parallel scan)
  P::prof(47);
  const uint32_t np = s.n_pend;
  for (uint32_t b = 0; b < np; b += 64) {
    int n = (int)amin<uint32_t>(64, np - b);
    uint64_t m = P::ballot(n, [&](int i) {
      const L1Pend& e = s.pend[b + i];
      return e.valid && e.line == line && (e.need & sectors) != 0;
    });
    while (m) {
      int i = ffs64(m);
      m &= m - 1;
      L1Pend& e = s.pend[b + i];
      e.need &= (uint8_t)~sectors;
      if (e.need) continue;
      e.valid = 0;
      sm_miss_access_done(s, c, e.warp, e.slot, now);
    }
  }
  // compact the pending table tail
  while (s.n_pend && !s.pend[s.n_pend - 1].valid) s.n_pend--;
  P::prof(41);
}

// ---------------------------------------------------------------------------
// L1 instruction cache (reference read_only_cache m_L1I: fetch probes it with
// the warp's next PC + PROGRAM_MEM_START, a miss parks the warp in
// imiss_pending until the line returns from L2, shader.cc:918-1020, 3989)
template <class P, class S>
SIM_HDI int il1_find(const S& s, const CacheGeom& g, uint32_t set, uint64_t line) {
  const L1Line* base = &s.il1[set * g.assoc];
  uint64_t m = P::ballot((int)amin<uint32_t>(g.assoc, 64), [&](int w) { return base[w].valid && base[w].tag == line; });
  return m ? ffs64(m) : -1;
}

template <class P, class S>
SIM_HDI void il1_fill(S& s, const SimCfg& c, uint64_t line) {
  const CacheGeom& g = c.il1;
  const uint32_t set = cache_set_index(g, line);
  if (il1_find<P>(s, g, set, line) < 0) {
    L1Line* base = &s.il1[set * g.assoc];
    const int v = P::argmin((int)amin<uint32_t>(g.assoc, 64), [&](int w) -> uint64_t {
      return base[w].valid ? (1ull << 40) | base[w].lru : (uint64_t)w;
    });
    base[v].tag = line;
    base[v].valid = 0xf;
    base[v].lru = ++s.l1_stamp;
  }
  const int mi = P::find_first((int)g.mshr_entries, [&](int i) -> bool { return s.imshr[i].valid && s.imshr[i].line == line; });
  if (mi >= 0) s.imshr[mi].valid = 0;
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  P::each(nw, [&](int w) {
    if ((s.w_flags[w] & WF_IMISS) && s.w_iline[w] == line) s.w_flags[w] &= (uint8_t)~WF_IMISS;
  });
  P::sync();
}

// probe the instruction cache for warp w's next fetch; true = instructions
// available this cycle
// sequential instruction prefetch: request the next inst_prefetch code lines
// that are neither cached nor pending (no waiter; the fill path is the demand
// one), as far as free MSHRs and the injection port allow
template <class P, class S>
SIM_HDI void il1_prefetch(S& s, const SimCfg& c, uint64_t line) {
  const CacheGeom& g = c.il1;
  for (uint32_t k = 1; k <= c.inst_prefetch; ++k) {
    const uint64_t l = line + 128ull * k;
    if (il1_find<P>(s, g, cache_set_index(g, l), l) >= 0) continue;
    if (P::find_first((int)g.mshr_entries, [&](int i) -> bool { return s.imshr[i].valid && s.imshr[i].line == l; }) >= 0)
      continue;
    const int mi = P::find_first((int)g.mshr_entries, [&](int i) -> bool { return !s.imshr[i].valid; });
    if (mi < 0 || !sm_can_send(s, c)) return;
    s.imshr[mi].valid = 1;
    s.imshr[mi].line = l;
    s.imshr[mi].merges = 0;
    s.imshr[mi].t_issue = 0;
    sm_send(s, c, P_RD, l, 0xf, 128, 0x40000000u | (uint32_t)mi);
    s.sadd(SK(il1_prefetch), 1);
  }
}

template <class P, class S>
SIM_HDI bool il1_fetch(S& s, const SimCfg& c, const KernelTab& kt, uint32_t w) {
  const CacheGeom& g = c.il1;
  const uint32_t pc = P::uni(s.w_win[w][P::uni((uint32_t)s.w_next[w]) & (kWin - 1)].pc);
  const uint64_t line = (kProgramMemStart + pc) & ~127ull;
  // fetch-block mode: w_iline holds the block the warp's last fetch read
  // (tagged with bit 0; a WF_IMISS warp's code line has it clear)
  const uint64_t blk = c.ifetch_block ? (((kProgramMemStart + pc) & ~(uint64_t)(c.ifetch_block - 1)) | 1ull) : 0;
  if (blk && P::uni((uint64_t)s.w_iline[w]) == blk) return true;
  const uint32_t set = cache_set_index(g, line);
  const int way = il1_find<P>(s, g, set, line);
  if (way >= 0) {
    if (g.repl == REPL_LRU) s.il1[set * g.assoc + way].lru = ++s.l1_stamp;
    s.sadd(SK(il1) + (IL1_HIT), 1);
    if (c.inst_prefetch && ((kProgramMemStart + pc) & 127u) < 8u) il1_prefetch<P>(s, c, line);  // entering a line
    if (blk) s.w_iline[w] = blk;
    return true;
  }
  int mi = P::find_first((int)g.mshr_entries, [&](int i) -> bool { return s.imshr[i].valid && s.imshr[i].line == line; });
  if (mi >= 0) {
    if (s.imshr[mi].merges >= g.mshr_merge) { s.sadd(SK(il1) + (IL1_RES_FAIL), 1); return false; }
    s.imshr[mi].merges++;
    s.sadd(SK(il1) + (IL1_MSHR_HIT), 1);
  } else {
    mi = P::find_first((int)g.mshr_entries, [&](int i) -> bool { return !s.imshr[i].valid; });
    if (mi < 0 || !sm_can_send(s, c)) { s.sadd(SK(il1) + (IL1_RES_FAIL), 1); return false; }
    s.imshr[mi].valid = 1;
    s.imshr[mi].line = line;
    s.imshr[mi].merges = 0;
    s.imshr[mi].t_issue = 0;
    sm_send(s, c, P_RD, line, 0xf, 128, 0x40000000u | (uint32_t)mi);
    s.sadd(SK(il1) + (IL1_MISS), 1);
    if (c.inst_prefetch) il1_prefetch<P>(s, c, line);
  }
  s.w_flags[w] |= WF_IMISS;
  s.w_iline[w] = line;
  return false;
}

// ---------------------------------------------------------------------------
// Crossbar output port (reference xbar_router::RR_Advance / iSLIP_Advance,
// local_interconnect.cc:123-270).  Arrivals reach a destination's port in
// time order (the sorted input queue); each cycle the port grants ONE of the
// inputs whose packet has arrived, in round-robin order from the arbiter's
// pointer -- the rotating global pointer (RR) or the per-output pointer moved
// past the granted input (iSLIP).  Input-side virtual output queues: a packet
// waiting for one busy output never blocks its input's packets to others
// (the sender's injection port already serialises one flit per cycle).
// Arbitration looks at the 64 oldest arrivals.
struct XbarGrant {
  uint32_t off;    // offset of the granted packet from the queue head
  uint32_t ready;  // inputs' packets ready at the port this cycle (>= 1)
};
template <class P>
SIM_HDI XbarGrant xbar_pick(const Pkt* q, uint32_t head, uint32_t n, uint32_t cap, uint64_t now_fs,
                            const SimCfg& c, uint64_t icnt_cycle, uint16_t& arb_next, uint16_t& arb_cnt,
                            uint32_t nsrc) {
  const uint32_t m = n < 64u ? n : 64u;
  const uint32_t ptr = c.icnt_arbiter ? (uint32_t)arb_next % nsrc : (uint32_t)(icnt_cycle % nsrc);
  // packets that reached the port (arrival order is only nearly time order:
  // serialised multi-flit packets can arrive after later-injected ones)
  const uint64_t rmask = P::ballot((int)m, [&](int i) { return q[(head + (uint32_t)i) % cap].t <= now_fs; });
  const uint32_t ready = (uint32_t)popc64(rmask);
  uint32_t off = rmask ? (uint32_t)ffs64(rmask) : 0u;
  if (ready > 1) {
    const int o = P::argmin((int)m, [&](int i) -> uint64_t {
      if (!(rmask >> i & 1ull)) return ~0ull;
      const Pkt& p = q[(head + (uint32_t)i) % cap];
      const uint32_t d = ((uint32_t)p.src + nsrc - ptr) % nsrc;
      return (uint64_t)d << 8 | (uint64_t)i;
    });
    off = o < 0 ? 0u : (uint32_t)o;
  }
  if (c.icnt_arbiter) {
    if (arb_cnt <= 1) {
      arb_next = (uint16_t)(((uint32_t)P::uni(q[(head + off) % cap].src) + 1) % nsrc);
      arb_cnt = (uint16_t)c.icnt_grant_cycles;
    } else {
      arb_cnt = (uint16_t)(arb_cnt - 1);
    }
  }
  return XbarGrant{off, ready ? ready : 1u};
}
// remove the packet at `off` from the head of a time-ordered ring (the
// packets before it move up one slot, keeping their order)
template <class Q>
SIM_HDI Pkt xbar_take(Q& q, uint32_t& head, uint32_t& n, uint32_t cap, uint32_t off) {
  const Pkt p = q[(head + off) % cap];
  for (uint32_t j = off; j > 0; --j) q[(head + j) % cap] = q[(head + j - 1) % cap];
  head = (head + 1) % cap;
  n--;
  return p;
}

// The reply path into the SM, one step per core cycle in the reference's
// order (simt_core_cluster::icnt_cycle runs before the core, shader.cc:4623-4660;
// ldst_unit::cycle consumes its response FIFO, shader.cc:2810-2857):
//   1. the head of the cluster ejection buffer moves to the LD/ST response
//      FIFO if that has room (an instruction-cache fill goes to the fetch
//      unit at once: accept_fetch_response);
//   2. one packet that reached the SM's crossbar output port is ejected into
//      the cluster buffer if it is not full (otherwise it waits in the port);
//   3. the LD/ST unit consumes the head of its response FIFO: store ack,
//      bypass / atomic load completion, or L1 fill.  A fill may evict a dirty
//      line whose write-back needs an injection-queue entry: with that queue
//      full the fill waits (like the reference's fill-port reservation)
//      instead of dropping the write-back.
template <class P, class S>
SIM_HDI void sm_receive(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  // 1. cluster buffer -> LD/ST response FIFO
  if (P::uni(s.cl_n)) {
    const uint32_t ch = P::uni(s.cl_head);
    const Pkt& h = s.rsp_cl[ch];
    const bool ifill = (P::uni(h.tag) & 0xc0000000u) == 0x40000000u && P::uni(h.type) != P_WR_ACK;
    if (ifill) {
      il1_fill<P>(s, c, P::uni(h.addr));
      s.cl_head = (ch + 1) % kEjectQ;
      s.cl_n = P::uni(s.cl_n) - 1;
    } else if (P::uni(s.ld_n) < c.ldst_resp_buf) {
      const uint32_t li = (P::uni(s.ld_head) + P::uni(s.ld_n)) % kLdstRespQ;
      const Pkt v = P::uni(h);
      P::one([&] { s.rsp_ld[li] = v; });
      s.ld_n = P::uni(s.ld_n) + 1;
      s.cl_head = (ch + 1) % kEjectQ;
      s.cl_n = P::uni(s.cl_n) - 1;
    }
  }
  // 2. crossbar output port -> cluster ejection buffer
  if (P::uni(s.inq_n) && P::uni(s.cl_n) < c.eject_buf &&
      P::uni(s.inq[P::uni(s.inq_head)].t) <= core_fs(c, now)) {
    Pkt q;
    uint32_t head = P::uni(s.inq_head), n = P::uni(s.inq_n);
    uint16_t an = s.arb_next, ac = s.arb_cnt;
    P::prof(40);
    const XbarGrant g = xbar_pick<P>(s.inq, head, n, kInQ, core_fs(c, now), c, fdiv(core_fs(c, now), c.dv_icnt),
                                     an, ac, c.n_subpart);
    P::prof(0);
    s.arb_next = an;
    s.arb_cnt = ac;
    s.sadd(SK(icnt_reply_conflicts), g.ready - 1);
    q = P::uni(xbar_take(s.inq, head, n, kInQ, g.off));
    s.sadd(SK(icnt_reply_queue_cycles), fdiv(core_fs(c, now) - q.t, c.dv_icnt));
    s.inq_head = head;
    s.inq_n = n;
    if (trace_sm_on(c, TS_INTERCONNECT, s.id)) P::one([&] { trace_put(c, s.id, now, EV_PKT_RECV, q.type, q.addr); });
    s.outstanding--;
    s.sadd(SK(pkts_in), 1);
    s.sadd(SK(bytes_in), q.size);
    const uint32_t ci = (P::uni(s.cl_head) + P::uni(s.cl_n)) % kEjectQ;
    P::one([&] { s.rsp_cl[ci] = q; });
    s.cl_n = P::uni(s.cl_n) + 1;
  }
  // 3. the LD/ST unit consumes one response
  if (!P::uni(s.ld_n)) return;
  if (P::uni(s.outq_n) >= (uint32_t)kOutQ) return;
  const uint32_t lh = P::uni(s.ld_head);
  const Pkt q = P::uni(s.rsp_ld[lh]);
  s.ld_head = (lh + 1) % kLdstRespQ;
  s.ld_n = P::uni(s.ld_n) - 1;
  if (q.type == P_WR_ACK) {
    if (!(q.tag & kTagL1Writeback)) {
      uint32_t w = q.tag & 0xff;
      s.w_stores[w]--;
    }
    s.last_progress = now;
  } else if (q.tag & 0x80000000u) {  // direct (bypass / atomic) load access
    uint32_t w = q.tag & 0xff, sl = (q.tag >> 8) & 0xff;
    sm_miss_access_done(s, c, w, sl, now);
  } else {
    P::prof(41);
    l1_fill<P>(s, x, q.addr, q.sectors, now);
    P::prof(0);
  }
}

// ---------------------------------------------------------------------------
// LD/ST unit: processes the coalesced accesses of one warp instruction
SIM_HDI uint32_t l1_stat_type(uint8_t space, bool write, bool atomic) {
  if (atomic) return L1T_ATOMIC;
  if (space == S_LOCAL) return write ? L1T_LOCAL_W : L1T_LOCAL_R;
  return write ? L1T_GLOBAL_W : L1T_GLOBAL_R;
}

template <class P, class S>
SIM_HDI void sm_ldst(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  LdstState& u = s.ldst;
  if (!P::uni(u.busy)) return;
  const TInst in = P::uni(u.inst);
  const uint32_t w = P::uni(u.warp);
  if (in.space == S_SHARED) {
    // bank-conflict serialisation: nacc == conflict degree (precomputed);
    // with -sim_lds_port_bytes the data path's cycles (ii, set at ingest)
    // bound it from below
    const uint32_t cdeg = in.width ? in.width : 1;
    const uint32_t deg = (c.lds_port_bytes && in.ii > cdeg) ? (uint32_t)in.ii : cdeg;
    if ((uint32_t)(now - P::uni(u.start)) + 1 < deg) return;
    uint8_t kind = (in.cls == OC_STORE) ? 1 : 0;
    if (!hit_push(s, now + c.smem_latency, (uint8_t)w, P::uni(u.slot), kind)) return;
    s.sadd(SK(shmem_acc), 1);
    s.sadd(SK(shmem_conflict_cycles), cdeg - 1);
    u.busy = 0;
    return;
  }
  const bool is_store = in.cls == OC_STORE;
  const bool atomic = (in.flags & F_ATOMIC) != 0;
  const CacheGeom g = l1_geom(c, s);
  // scalar loads always use the (scalar) cache, -gpgpu_gmem_skip_L1D aside
  const bool bypass = atomic || (in.flags & F_BYPASS_L1) || (c.gmem_skip_l1 && in.space != S_CONST) || g.disabled;
  const uint32_t nacc = in.width;
  const uint32_t stype = l1_stat_type(in.space, is_store, atomic);
  uint32_t banks_used = 0;
  uint32_t processed = 0;
  uint32_t unext = P::uni(u.next);
  const uint8_t uslot = P::uni(u.slot);
  // access records were brought into the unit at dispatch
  P::fetch_wait();
  const bool port = c.l1_port_bytes && in.space != S_CONST;
  while (unext < nacc && processed < c.l1_banks) {
    const TAcc a = P::uni(s.ldst_acc[unext]);
    uint32_t bbit = 1u << (a.bank & 31);
    if (banks_used & bbit) break;  // L1 bank conflict: next cycle
    // L1 data path busy (-sim_l1_port_bytes): the access waits
    if (port && (int32_t)(P::uni(u.port_free) - (uint32_t)now) > 0) break;
    if (c.perfect_mem) {
      // ideal memory: loads/atomics return after the L1 latency, stores retire at once
      if (!is_store) {
        if (!hit_push(s, now + c.l1_latency, (uint8_t)w, uslot, 0)) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
      }
      SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_HIT, 1);
    } else if (is_store) {
      // write policy (reference data_cache wr_hit_* / wr_miss_*,
      // gpu-cache.cc:1229-1599); 'L' = write-back for local, write-evict for
      // global data (wr_hit_global_we_local_wb)
      uint8_t pol = g.wpolicy;
      if (pol == WP_LOCAL_WB_GLOBAL_WT) pol = in.space == S_LOCAL ? WP_WRITE_BACK : WP_WRITE_EVICT;
      if (bypass || pol == WP_READ_ONLY) {
        if (!sm_can_send_n(s, c, wr_packets<S>(c, a.sectors))) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
        s.w_stores[w] += sm_send_write(s, c, a.line, a.sectors, a.bytes, w);
        SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_BYPASS, 1);
      } else {
        const uint32_t set = cache_set_index(g, a.line);
        int way = l1_find<P>(s, g, set, a.line);
        const uint8_t have = way >= 0 ? P::uni(s.l1[set * g.assoc + way].valid) : (uint8_t)0;
        const bool hit = way >= 0 && (have & a.sectors) == a.sectors;
        // a write covering whole sectors leaves them readable (lazy / fetch-on-write)
        const bool full = g.sectored ? a.bytes >= 32u * (uint32_t)popc64(a.sectors) : a.bytes >= g.line;
        const bool wb = pol == WP_WRITE_BACK;
        const uint8_t wa = g.walloc;
        if (hit) {
          if (wb) {
            // write-back hit: the line absorbs the store, nothing goes below
            L1Line& L = s.l1[set * g.assoc + way];
            L.dirty |= a.sectors;
            if (g.repl == REPL_LRU) L.lru = ++s.l1_stamp;
          } else {
            if (!sm_can_send_n(s, c, wr_packets<S>(c, a.sectors))) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
            s.w_stores[w] += sm_send_write(s, c, a.line, a.sectors, a.bytes, w);
            L1Line& L = s.l1[set * g.assoc + way];
            if (pol == WP_WRITE_EVICT) L.valid &= (uint8_t)~a.sectors;
            else if (g.repl == REPL_LRU) L.lru = ++s.l1_stamp;
          }
          SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_HIT, 1);
        } else if (wa == 'N' || pol == WP_WRITE_EVICT) {
          // no write-allocate: straight to the L2
          if (!sm_can_send_n(s, c, wr_packets<S>(c, a.sectors))) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
          s.w_stores[w] += sm_send_write(s, c, a.line, a.sectors, a.bytes, w);
          if (way >= 0 && pol == WP_WRITE_EVICT) s.l1[set * g.assoc + way].valid &= (uint8_t)~a.sectors;
          SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_MISS, 1);
        } else {
          // write-allocate: lazy fetch on read ('L'), fetch-on-write ('F'),
          // naive ('W': write and read the line)
          const bool fetch = wa == 'W' || (wa == 'F' && !full);
          const bool send_wr = !wb || wa == 'W';
          int mi = -1;
          if (fetch) mi = P::find_first((int)c.l1.mshr_entries, [&](int i) -> bool { return s.mshr[i].valid && s.mshr[i].line == a.line; });
          const int mfree = fetch && mi < 0 ? P::find_first((int)c.l1.mshr_entries, [&](int i) -> bool { return !s.mshr[i].valid; }) : 0;
          const uint32_t need = (send_wr ? wr_packets<S>(c, a.sectors) : 0u) + (fetch ? 1u : 0u) + 1u;  // + a possible dirty victim
          if (!sm_can_send_n(s, c, need) || mfree < 0) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
          if (send_wr) s.w_stores[w] += sm_send_write(s, c, a.line, a.sectors, a.bytes, w);
          if (way < 0) {
            way = l1_victim<P>(s, g, set);
            l1_evict<P>(s, c, set * g.assoc + way);
            L1Line& L = s.l1[set * g.assoc + way];
            L.tag = a.line;
            L.valid = 0;
            L.dirty = 0;
            L.lru = ++s.l1_stamp;
          }
          L1Line& L = s.l1[set * g.assoc + way];
          if (full && !fetch) L.valid |= a.sectors;
          if (wb) L.dirty |= a.sectors;
          if (g.repl == REPL_LRU) L.lru = ++s.l1_stamp;
          if (fetch) {
            // read the written line's missing sectors (no waiter: the fill
            // only makes them readable)
            const uint8_t want = a.sectors & (uint8_t)~P::uni(L.valid);
            if (mi < 0) {
              mi = mfree;
              s.mshr[mi].valid = 1;
              s.mshr[mi].line = a.line;
              s.mshr[mi].requested = 0;
              s.mshr[mi].merges = 0;
              s.mshr[mi].t_issue = (uint32_t)now;
            }
            const uint8_t req = want & (uint8_t)~P::uni(s.mshr[mi].requested);
            if (req) {
              s.mshr[mi].requested |= req;
              sm_send(s, c, P_RD, a.line, req, (uint16_t)(32 * popc64(req)), (uint32_t)mi);
            }
          }
          SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_MISS, 1);
        }
      }
    } else if (bypass) {
      if (!sm_can_send(s, c)) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
      uint32_t tag = 0x80000000u | ((uint32_t)uslot << 8) | w;
      sm_send(s, c, atomic ? P_ATOM : P_RD, a.line, a.sectors, a.bytes, tag);
      SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_BYPASS, 1);
    } else {
      P::prof(36);
      uint32_t set = cache_set_index(g, a.line);
      int way = l1_find<P>(s, g, set, a.line);
      uint8_t have = way >= 0 ? s.l1[set * g.assoc + way].valid : 0;
      uint8_t miss = a.sectors & (uint8_t)~have;
      P::prof(3);
      if (miss == 0) {
        P::prof(46);
        const bool pushed = hit_push(s, now + c.l1_latency, (uint8_t)w, uslot, 0);
        P::prof(3);
        if (!pushed) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
        if (g.repl == REPL_LRU) s.l1[set * g.assoc + way].lru = ++s.l1_stamp;
        SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_HIT, 1);
      } else {
        if (s.n_pend >= (uint32_t)kMaxPend) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
        P::prof(37);
        int mi = P::find_first((int)c.l1.mshr_entries, [&](int i) -> bool { return s.mshr[i].valid && s.mshr[i].line == a.line; });
        P::prof(3);
        // a sectored L1 ('S') fetches the sectors the access misses; a
        // line-granular one ('N') the whole line it does not hold (the L2's
        // 'N' fill, mem.h l2_access)
        const uint8_t fetch = g.sectored ? miss : (uint8_t)(0xFu & ~have);
        uint8_t need_req = fetch;
        if (mi >= 0) need_req = fetch & (uint8_t)~s.mshr[mi].requested;
        bool merged = (mi >= 0 && need_req == 0);
        if (merged) {
          if (s.mshr[mi].merges >= c.l1.mshr_merge) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
          s.mshr[mi].merges++;
          SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_MSHR_HIT, 1);
        } else {
          if (!sm_can_send(s, c)) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
          if (mi < 0) {
            P::prof(37);
            mi = P::find_first((int)c.l1.mshr_entries, [&](int i) -> bool { return !s.mshr[i].valid; });
            P::prof(3);
            if (mi < 0) { SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_RES_FAIL, 1); break; }
            s.mshr[mi].valid = 1;
            s.mshr[mi].line = a.line;
            s.mshr[mi].requested = 0;
            s.mshr[mi].merges = 0;
            s.mshr[mi].t_issue = (uint32_t)now;
          }
          s.mshr[mi].requested |= need_req;
          P::prof(39);
          sm_send(s, c, P_RD, a.line, need_req, a.bytes, (uint32_t)mi);
          P::prof(3);
          SADD_IN(s, l1, L1T_COUNT * L1O_COUNT, (stype) * L1O_COUNT + L1O_MISS, 1);
        }
        // register the waiter (first free entry)
        P::prof(38);
        uint32_t pi = s.n_pend;
        for (uint32_t b = 0; b < s.n_pend; b += 64) {
          int n = (int)amin<uint32_t>(64, s.n_pend - b);
          uint64_t m = P::ballot(n, [&](int i) { return !s.pend[b + i].valid; });
          if (m) { pi = b + ffs64(m); break; }
        }
        L1Pend& e = s.pend[pi];
        e.line = a.line;
        e.need = miss;
        e.warp = (uint8_t)w;
        e.slot = uslot;
        e.valid = 1;
        if (pi == s.n_pend) s.n_pend++;
        P::prof(3);
      }
    }
    if (in.space != S_CONST)
      s.sadd(SK(l1_lookups64), (uint32_t)((a.sectors & 3u) != 0) + (uint32_t)((a.sectors & 12u) != 0));
    if (port) {
      // the access's bytes cross the data path (hit data, store data, or the
      // miss's fill later: charged here, once per access)
      const uint32_t pf = P::uni(u.port_free);
      const uint32_t from = (int32_t)(pf - (uint32_t)now) > 0 ? pf : (uint32_t)now;
      uint32_t pb = a.bytes ? a.bytes : 1u;
      if (c.l1_port_granule == 32) pb = 32u * (uint32_t)popc64(a.sectors);
      else if (c.l1_port_granule == 64) pb = 64u * (((a.sectors & 3u) != 0) + ((a.sectors & 12u) != 0));
      u.port_free = from + (pb + c.l1_port_bytes - 1) / c.l1_port_bytes;
    }
    banks_used |= bbit;
    unext++;
    u.next = (uint8_t)unext;
    processed++;
  }
  if (unext >= nacc) {
    if (is_store) {
      s.w_inflight[w]--;  // store instruction leaves the pipeline; acks tracked in w_stores
      s.last_progress = now;
    }
    u.busy = 0;
  }
}

// ---------------------------------------------------------------------------
// operand collectors -> functional units
SIM_HDI uint32_t reg_bank(const SimCfg& c, uint32_t sched, uint32_t warp, uint32_t reg) {
  uint32_t nb = c.reg_banks ? c.reg_banks : 1;
  uint32_t per = (c.sub_core && c.n_sched) ? (nb / c.n_sched ? nb / c.n_sched : 1) : nb;
  uint32_t base = (c.sub_core && c.n_sched) ? (sched * per) % nb : 0;
  // power-of-two bank groups (every tested config) avoid integer division
  if ((per & (per - 1)) == 0) return base + ((reg + warp) & (per - 1));
  return base + (reg + warp) % per;
}

// operand reads: each register bank serves one read per round, up to
// reg_port_tp rounds per cycle, oldest collector first.  The reference's
// arbiter (opndcoll_rfu_t::allocate_reads, shader.cc:3650-3733) is replaced by
// the equivalent greedy pass: the oldest collector with a grantable operand
// keeps winning until it has none left (banks only become busy within a
// round), so the round visits collectors once in age order, each taking its
// operands on free banks in operand order, at most `noc` grants per round.
template <class P, class S>
SIM_HDI void sm_read_operands(S& s, const SimCfg& c) {
  uint32_t rmask = P::uni(s.oc_read_mask);
  if (!rmask) return;
  const int noc = (int)amin<uint32_t>(c.oc_units, kMaxOC);
  for (uint32_t round = 0; round < c.reg_port_tp && rmask; ++round) {
    const uint32_t want = rmask;
    const int nwant = popc64(want);
    const uint64_t ord = nwant == 1 ? (uint64_t)ffs64(want)
                                    : P::order16(noc, want, [&](int i) -> uint32_t { return s.oc_age[i]; });
    uint32_t bank_busy = 0, grants = 0;
    for (int r = 0; r < nwant && grants < (uint32_t)noc; ++r) {
      const int i = (int)((ord >> (4 * r)) & 15u);
      uint64_t b = P::uni((uint64_t)s.oc_banks[i]);
      uint32_t nr = (uint32_t)(b >> 40) & 0xffu;
      uint32_t got = 0;
      for (int j = 0; j < 5 && grants < (uint32_t)noc; ++j) {
        const uint32_t bj = (uint32_t)(b >> (8 * j)) & 0xffu;
        if (bj != 0xffu && !(bank_busy >> bj & 1u)) {
          bank_busy |= 1u << bj;
          b |= 0xffull << (8 * j);
          ++got;
          ++grants;
        }
      }
      if (got) {
        nr -= got;
        b = (b & ~(0xffull << 40)) | ((uint64_t)nr << 40);
        s.oc_banks[i] = b;
        s.sadd(SK(rf_reads), got);
        if (nr == 0) rmask &= ~(1u << i);
      }
      if (nr) s.sadd(SK(oc_bank_conflicts), nr);  // reads left waiting on a busy bank this round
    }
    s.oc_read_mask = rmask;
  }
}

// collectors whose operands are all read go to their unit, oldest first
template <class P, class S>
SIM_HDI void sm_dispatch(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  const KernelTab* x_kt = x.kt;
  const int noc = (int)amin<uint32_t>(c.oc_units, kMaxOC);
  const uint32_t wbw = wb_width(c);
  const uint32_t ready = P::uni(s.oc_mask & ~s.oc_read_mask);
  if (!ready) return;
  const int n = popc64(ready);
  const uint64_t ord =
      n == 1 ? (uint64_t)ffs64(ready) : P::order16(noc, ready, [&](int i) -> uint32_t { return s.oc_age[i]; });
  for (int r = 0; r < n; ++r) {
    const int best = (int)((ord >> (4 * r)) & 15u);
    const uint64_t info = P::uni((uint64_t)s.oc_info[best]);
    const uint32_t u = (uint32_t)(info >> 16) & 0xffu;
    if (u == U_MEM) {
      if (P::uni(s.ldst.busy)) continue;
      const TInst li = P::uni(s.oc_inst[best]);
      s.ldst.inst = li;
      s.ldst.busy = 1;
      s.ldst.warp = (uint8_t)(info & 0xffu);
      if (li.space != S_SHARED && li.width && li.mem != kNoMem) {
        // the warp's kernel's access table (slot in the top bits of its stream index)
        const KernelDesc& kacc = x_kt->k[P::uni((uint32_t)s.w_end[info & 0xffu]) >> kSlotShift];
        const TAcc* accs = kacc.accs;
        P::fetch_copy(&s.ldst_acc[0], &accs[li.mem & kacc.amask], (int)amin<uint32_t>(li.width, kMaxAccess));
      }
      s.ldst.slot = (uint8_t)((info >> 24) & 0xffu);  // load slot allocated at issue
      s.ldst.next = 0;
      s.ldst.start = (uint32_t)now;
      if (c.l1_addr_lanes && li.space != S_SHARED && li.space != S_CONST && li.width) {
        // the address stage takes the instruction's active lanes at
        // l1_addr_lanes per cycle before its first access reaches the data path
        const uint32_t pf = P::uni(s.ldst.port_free);
        const uint32_t from = (int32_t)(pf - (uint32_t)now) > 0 ? pf : (uint32_t)now;
        s.ldst.port_free = from + ((uint32_t)popc64(li.mask) + c.l1_addr_lanes - 1) / c.l1_addr_lanes;
      }
      s.sadd(SK(mem_insn), 1);
      s.oc_mask &= ~(1u << best);
      continue;
    }
    const uint32_t sched = (uint32_t)(info >> 8) & 0xffu;
    const uint32_t cnt = c.unit_count[u] ? c.unit_count[u] : 1;
    uint32_t phys = sched < cnt ? sched : sched % cnt;
    if (phys >= (uint32_t)kMaxSched) phys %= kMaxSched;
    const uint32_t fi = u * (uint32_t)kMaxSched + phys;
    const uint32_t nf = P::uni((uint32_t)s.fu_next[fi]);
    if ((int32_t)(nf - (uint32_t)now) > 0) continue;  // initiation interval
    uint32_t lat = (uint32_t)(info >> 32) & 0xffffu;
    if (!lat) lat = 1;
    if (lat >= (uint32_t)kWbRing) lat = kWbRing - 1;
    const uint32_t slot = (uint32_t)((now + lat) % kWbRing);
    const uint32_t nwb = P::uni(s.wb_cnt[slot]);
    if (nwb >= wbw) { s.sadd(SK(pipe_stall), 1); continue; }  // result bus busy
    s.wb_cnt[slot] = (uint8_t)(nwb + 1);
    const uint64_t bk = P::uni((uint64_t)s.oc_banks[best]);
    WbEnt& e = s.wb[slot][nwb];
    s.wb_occ[slot >> 6] |= 1ull << (slot & 63);
    e.warp = (uint8_t)(info & 0xffu);
    e.dst0 = (uint8_t)(bk >> 48);
    e.dst1 = (uint8_t)(bk >> 56);
    e.pad = 0;
    const uint32_t ii = (uint32_t)(info >> 48) & 0xffu;
    s.fu_next[fi] = (uint32_t)now + (ii ? ii : 1);
    s.oc_mask &= ~(1u << best);
  }
}

template <class P, class S>
SIM_HDI void sm_alloc_collectors(S& s, const SimCfg& c) {
  const int noc = (int)amin<uint32_t>(c.oc_units, kMaxOC);
  const uint32_t nsched = c.n_sched;
  const uint32_t per = (c.sub_core && nsched) ? (noc / nsched ? noc / nsched : 1) : (uint32_t)noc;
  // visit pending pipeline registers in (scheduler, unit) order via the mask
  uint64_t pend = P::uni(s.idoc_mask);
  uint32_t ocm = P::uni(s.oc_mask);
  while (pend) {
    const int bit = ffs64(pend);
    pend &= pend - 1;
    const uint32_t sc = (uint32_t)bit / U_COUNT, u = (uint32_t)bit % U_COUNT;
    // free collector in this scheduler's group
    uint32_t lo = c.sub_core ? (sc * per) % noc : 0;
    uint32_t hi = c.sub_core ? lo + per : (uint32_t)noc;
    if (hi > (uint32_t)noc) hi = noc;
    const uint32_t grp = ((hi >= 32 ? 0xffffffffu : ((1u << hi) - 1)) & ~((1u << lo) - 1));
    const uint32_t freem = grp & ~ocm;
    if (!freem) continue;
    const int f = ffs64(freem);
    ocm |= 1u << f;
    s.oc_mask = ocm;
    const uint64_t meta = P::uni((uint64_t)s.idoc_meta[bit]);
    const TInst rin = P::uni(s.idoc_inst[bit]);
    const uint32_t rw = (uint32_t)(meta & 0xffu);
    s.oc_inst[f] = rin;
    uint64_t bk = 0;
    uint32_t nread = 0;
    for (int j = 0; j < 5; ++j) {
      const uint8_t reg = rin.src[j];
      const uint32_t bank = reg ? reg_bank(c, sc, rw, reg - 1u) : 0xffu;
      bk |= (uint64_t)(bank & 0xffu) << (8 * j);
      nread += reg ? 1u : 0u;
    }
    bk |= (uint64_t)nread << 40 | (uint64_t)rin.dst[0] << 48 | (uint64_t)rin.dst[1] << 56;
    s.oc_banks[f] = bk;
    s.oc_info[f] = (uint64_t)rw | (uint64_t)sc << 8 | (uint64_t)u << 16 | ((meta >> 8) & 0xffull) << 24 |
                   (uint64_t)rin.lat << 32 | (uint64_t)rin.ii << 48;
    s.oc_age[f] = (uint32_t)(meta >> 32);
    if (nread) s.oc_read_mask |= 1u << f;
    s.idoc_mask &= ~(1ull << bit);
  }
}

// ---------------------------------------------------------------------------
// issue
template <class P, class S>
SIM_HDI void sm_barrier_check(S& s, uint32_t cta) {
  uint32_t live = s.cta_live[cta] - s.cta_nexit[cta];
  if (s.cta_bar[cta] > 0 && s.cta_bar[cta] >= live) {
    const uint32_t base = s.cta_wbase[cta], nw = s.cta_nw[cta];
    for (uint32_t w = base; w < base + nw && w < (uint32_t)kMaxWarps; ++w)
      s.w_flags[w] &= (uint8_t)~WF_BARRIER;
    s.cta_bar[cta] = 0;
  }
}

// x mod n for the small operands of the issue stage (x < 2n in the common
// case): a compare-and-subtract instead of an integer division on the GPU
SIM_HDI uint32_t mod_small(uint32_t x, uint32_t n) {
  if (x < n) return x;
  x -= n;
  return x < n ? x : x % n;
}
// the scheduler supervising warp w (w % n_sched; power-of-two counts mask)
SIM_HDI uint32_t sched_of(uint32_t w, uint32_t nsched) {
  return (nsched & (nsched - 1)) == 0 ? (w & (nsched - 1)) : w % nsched;
}

// can warp `w` issue its next instruction this cycle (scoreboard, flags,
// pipeline register and load slot availability)
template <class S>
SIM_HDI bool warp_sb_ok(const S& s, int w, const TInst& in) {
  for (int j = 0; j < 5; ++j)
    if (sbt(s.w_sb, w, in.src[j])) return false;
  return !sbt(s.w_sb, w, in.dst[0]) && !sbt(s.w_sb, w, in.dst[1]);
}
// warp_can_issue_i without the scoreboard test (warp_sb_ok)
template <class S>
SIM_HDI bool warp_can_issue_nosb(const S& s, const SimCfg& c, int w, const TInst& in, uint32_t nsched,
                                 uint64_t idoc_busy) {
  uint8_t f = s.w_flags[w];
  if (!(f & WF_ACTIVE) || (f & (WF_EXITING | WF_BARRIER | WF_MEMBAR | WF_WAITCNT))) return false;
  if (s.w_ibuf[w] == 0) return false;
  uint32_t u = unit_of(c, in.cls);
  uint32_t sc = sched_of((uint32_t)w, nsched);
  if (in.cls == OC_EXIT || in.cls == OC_BARRIER || in.cls == OC_MEMBAR || in.cls == OC_NOP || (in.flags & F_WAITCNT))
    return true;  // handled at issue, no pipeline register needed
  if (idoc_busy >> (sc * U_COUNT + u) & 1ull) return false;
  if (u == U_MEM && in.cls == OC_LOAD && s.w_slot_used[w] == 0xff) return false;
  return true;
}
template <class S>
SIM_HDI bool warp_can_issue_i(const S& s, const SimCfg& c, int w, const TInst& in, uint32_t nsched,
                              uint64_t idoc_busy) {
  return warp_can_issue_nosb(s, c, w, in, nsched, idoc_busy) && warp_sb_ok(s, w, in);
}
template <class S>
SIM_HDI bool warp_can_issue(const S& s, const SimCfg& c, const KernelTab& kt, int w, uint32_t nsched,
                            uint64_t idoc_busy) {
  if (!(s.w_flags[w] & WF_ACTIVE) || s.w_ibuf[w] == 0) return false;
  const TInst in = s.w_win[w][s.w_head[w] & (kWin - 1)];  // ibuf > 0: the head is in the window
  return warp_can_issue_i(s, c, w, in, nsched, idoc_busy);
}

// -gpgpu_warp_issue_interval: has the warp's issue interval elapsed at `now`
template <class S>
SIM_HDI bool warp_issue_due(const S& s, const SimCfg& c, int w, uint64_t now) {
  return c.warp_issue_interval <= 1 || now >= s.w_issue_ok[w];
}

// issue one instruction `in` (trace index hidx) of warp w from scheduler sc;
// returns its execution unit, or -1 for the kinds handled at issue (EXIT,
// barrier, fence, waitcnt, NOP)
template <class P, class S>
SIM_HDI int sm_issue_one(S& s, const SmCtx& x, uint64_t now, uint32_t sc, uint32_t w, const TInst& in,
                         uint32_t hidx) {
  const SimCfg& c = *x.cfg;
  if (trace_sm_on(c, TS_WARP_SCHEDULER, s.id))
    P::one([&] { trace_put(c, s.id, now, EV_ISSUE, (uint16_t)w, (uint64_t)in.pc | (uint64_t)in.opcode << 32); });
  s.w_head[w] = hidx + 1;
  s.w_ibuf[w] = (uint8_t)(P::uni((uint8_t)s.w_ibuf[w]) - 1);
  // stats: instruction counts at issue (reference counts active threads,
  // shader.cc:1911)
  s.sadd(SK(warp_insn), 1);
  s.sadd(SK(thread_insn), (uint64_t)popc64(in.mask));
  SADD_IN(s, cls_insn, OC_COUNT, in.cls < OC_COUNT ? in.cls : OC_ALU, 1);
  SADD_IN(s, sq_insn, 8, sq_class(in), 1);
  // LDC / s_load: an ALU-timed instruction with a constant-cache operand
  // (reference trace_driven.cc:255-261 keeps LDC an ALU op; shader.cc:3287)
  if (in.space == S_CONST) s.sadd(SK(power_acc) + PWR_CONST_OPERAND, 1);
  // per-issue energy: the instruction's active lanes on its unit kind (the
  // scalar unit executes once per wave)
  {
    const uint32_t pk = (uint32_t)(in.flags >> 4);
    if (pk) SADD_IN(s, power_acc, 16, pk, pk == PWR_SALU ? 1ull : (uint64_t)popc64(in.mask));
  }
  s.last_progress = now;
  const uint32_t cta = P::uni((uint8_t)s.w_cta[w]);
  if (in.cls == OC_EXIT) {
    // lanes retire; the warp ends only when EXIT is its last instruction
    // (reference checkExecutionStatusAndUpdate, trace_driven.cc:588-606)
    if (hidx + 1 >= P::uni((uint32_t)s.w_end[w])) {
      s.w_flags[w] |= WF_EXITING;
      s.cta_nexit[cta]++;
      sm_barrier_check<P>(s, cta);
    }
    return -1;
  }
  if (in.cls == OC_BARRIER) {
    s.w_flags[w] |= WF_BARRIER;
    s.cta_bar[cta]++;
    sm_barrier_check<P>(s, cta);
    return -1;
  }
  if (in.cls == OC_MEMBAR) {
    if (s.w_stores[w]) {
      s.w_flags[w] |= WF_MEMBAR;
      s.n_wait_flags++;
    }
    return -1;
  }
  if (in.flags & F_WAITCNT) {
    s.w_wait[w] = in.lat;
    if (!waitcnt_met(s, w)) {
      s.w_flags[w] |= WF_WAITCNT;
      s.n_wait_flags++;
    }
    return -1;
  }
  if (in.cls == OC_NOP) return -1;
  const uint32_t u = unit_of(c, in.cls);
  const uint32_t kk = sc * U_COUNT + u;
  TInst ri = in;
  uint32_t lslot = 0xff;
  s.w_inflight[w]++;
  if (in.cls == OC_LOAD) {
    // allocate a load slot; scoreboard reserves destination registers
    uint8_t used = P::uni((uint8_t)s.w_slot_used[w]);
    uint32_t sl = (uint32_t)ffs64((uint64_t)(uint8_t)~used);
    s.w_slot_used[w] = (uint8_t)(used | (1u << sl));
    s.w_loads[w]++;
    uint32_t nacc = (in.space == S_SHARED) ? 1u : (uint32_t)in.width;
    if (nacc == 0) nacc = 1;
    s.w_slot_pend[w][sl] = (uint16_t)nacc;
    s.w_slot_dst[w][sl][0] = in.dst[0];
    s.w_slot_dst[w][sl][1] = in.dst[1];
    lslot = sl;
    if (in.space != S_SHARED && in.width == 0) {
      // memory instruction without any active access: completes via ring
      s.w_slot_pend[w][sl] = 1;
      ri.space = S_SHARED;
      ri.width = 1;
    }
    // slots lgkmcnt counts: LDS and scalar (SMEM) loads
    if (ri.space == S_SHARED || ri.space == S_CONST) s.w_slot_lds[w] = (uint8_t)(s.w_slot_lds[w] | (1u << sl));
  } else if (in.cls == OC_STORE && in.space != S_SHARED && in.width == 0) {
    ri.space = S_SHARED;
    ri.width = 1;
  }
  if (in.cls == OC_STORE && ri.space == S_SHARED) s.w_lds_st[w]++;
  s.idoc_inst[kk] = ri;
  s.idoc_meta[kk] = idoc_pack(w, lslot, ++s.age_ctr);
  s.idoc_mask |= 1ull << kk;
  sbs(s.w_sb, w, in.dst[0]);
  sbs(s.w_sb, w, in.dst[1]);
  return (int)u;
}

// does `in` read a register that an in-flight load of warp w will write (the
// reference scoreboard's long-operation test, Scoreboard::islongop)
template <class S>
SIM_HDI bool waits_long_op(const S& s, int w, const TInst& in) {
  const uint8_t used = s.w_slot_used[w];
  for (int sl = 0; sl < kLoadSlots; ++sl) {
    if (!(used >> sl & 1u)) continue;
    for (int d = 0; d < 2; ++d) {
      const uint8_t r = s.w_slot_dst[w][sl][d];
      if (!r) continue;
      for (int j = 0; j < 5; ++j)
        if (in.src[j] == r) return true;
    }
  }
  return false;
}

// warps with a valid instruction (buffered, not parked, issue interval
// elapsed) and, among them, those whose operands are ready (the reference
// scheduler_unit::cycle's valid_inst / ready_inst, shader.cc:1547-1555)
template <class P, class S>
SIM_HDI void sm_stall_masks(const S& s, const SimCfg& c, uint64_t now, uint64_t live, uint64_t& valid_m,
                            uint64_t& sbok_m) {
  valid_m = P::ballot_m(live, [&](int w) -> bool {
    const uint8_t f = s.w_flags[w];
    return (f & WF_ACTIVE) && !(f & (WF_EXITING | WF_BARRIER | WF_MEMBAR | WF_WAITCNT)) && s.w_ibuf[w] != 0 &&
           warp_issue_due(s, c, w, now);
  });
  sbok_m = P::ballot_m(valid_m, [&](int w) -> bool {
    const TInst& in = s.w_win[w][s.w_head[w] & (kWin - 1)];
    for (int j = 0; j < 5; ++j)
      if (sbt(s.w_sb, w, in.src[j])) return false;
    return !sbt(s.w_sb, w, in.dst[0]) && !sbt(s.w_sb, w, in.dst[1]);
  });
}
// stall class of one scheduler without an issue (issue_distro index 0..2)
SIM_HDI uint32_t stall_class(uint64_t mine, uint64_t valid_m, uint64_t sbok_m) {
  return !(valid_m & mine) ? 0u : !(sbok_m & mine) ? 1u : 2u;
}

// the scheduler picks of one cycle for the policies whose pick depends only
// on the ready mask and the scheduler's own state (shared by both issue
// paths): returns the picked warp, or -1
template <class P, class S>
SIM_HDI int sched_pick(const S& s, const SimCfg& c, uint64_t now, int nw, uint64_t cand, uint32_t last) {
  switch (c.sched_policy) {
    case SCHED_GTO:
      if (last < (uint32_t)nw && (cand >> last & 1ull)) return (int)last;
      [[fallthrough]];
    case SCHED_OLDEST:
      return P::argmin(nw, [&](int w) -> uint64_t {
        return (cand >> w & 1ull) ? ((uint64_t)s.w_age[w] << 8 | (uint64_t)w) : ~0ull;
      });
    case SCHED_RRR: {
      uint32_t start = (uint32_t)(now % (uint64_t)nw);
      uint64_t r = rotr64(cand, start, (unsigned)nw);
      return (int)mod_small((uint32_t)ffs64(r) + start, (uint32_t)nw);
    }
    default: {  // LRR: first ready warp after the last issued one
      uint32_t start = mod_small(last + 1, (uint32_t)nw);
      uint64_t r = rotr64(cand, start, (unsigned)nw);
      return (int)mod_small((uint32_t)ffs64(r) + start, (uint32_t)nw);
    }
  }
}

SIM_HDI bool issue_special(const TInst& in) {
  return in.cls == OC_EXIT || in.cls == OC_BARRIER || in.cls == OC_MEMBAR || in.cls == OC_NOP || (in.flags & F_WAITCNT);
}

// Lane-parallel issue (LRR / GTO / oldest / RRR, one instruction per warp per
// cycle, no scheduler trace stream).  The schedulers pick exactly as in the
// sequential loop below; then the picked warps issue together: lane w
// applies its own warp's bookkeeping (stream position, instruction buffer,
// in-flight count, load slot, scoreboard) instead of one scheduler after
// another in wave-uniform code.  The result equals the sequential loop's:
// schedulers own disjoint warps and ID_OC registers, the pipeline-register
// ages are ranked in scheduler order, the statistics are sums, and the
// instructions handled at issue (EXIT, barrier, fence, waitcnt, NOP -- they
// touch CTA state shared by the schedulers) run afterwards, in scheduler
// order, through sm_issue_one; they share no state with the pipeline issues.
// (Reference scheduler_unit::cycle, shader.cc:1249-1556, runs the
// schedulers one after another; so does sm_issue below for the other
// policies.)
template <class P, class S, class H>
SIM_HDI void sm_issue_par(S& s, const SmCtx& x, uint64_t now, const H& head, uint64_t ready, uint64_t live,
                          uint64_t sbok_all) {
  const SimCfg& c = *x.cfg;
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const uint32_t nsched = c.n_sched ? c.n_sched : 1;
  uint32_t n_idle = 0, idle_sc = 0, first_idle = nsched;
  uint64_t picks = 0;
  uint32_t pk_of = 0xffffffffu;  // byte sc: the warp scheduler sc picked (0xff: none)
  P::prof(48);
  for (uint32_t sc = 0; sc < nsched; ++sc) {
    const uint64_t mine = c.sched_mask[sc];
    const uint64_t cand = ready & mine;
    if (!cand) {
      if (live & mine) {
        ++n_idle;
        idle_sc |= 1u << sc;
        if (first_idle == nsched) first_idle = sc;
      }
      continue;
    }
    const uint32_t last = P::uni((uint32_t)s.sched_last[sc]);
    const uint32_t w = P::uni((uint32_t)sched_pick<P>(s, c, now, nw, cand, last));
    s.sched_last[sc] = w;
    if (c.warp_issue_interval > 1) P::one([&] { s.w_issue_ok[w] = now + c.warp_issue_interval; });
    pk_of = (pk_of & ~(0xffu << (8 * sc))) | w << (8 * sc);
    picks |= 1ull << w;
  }
  // Stall classes of the idle schedulers.  The sequential loop classifies at
  // its first idle scheduler, after the schedulers before it have issued --
  // their EXIT / barrier / fence instructions (step 3) can change the flags of
  // other schedulers' warps -- and before the ones after it: the same point
  // here, inside step 3's scheduler-order walk.  (The pipeline issues of
  // steps 1-2 touch only the issuing scheduler's own warps.)
  bool classified = n_idle == 0;
  auto classify = [&]() {
    classified = true;
    P::prof(49);
    // the scoreboard half from before the issues (sbok_all): a scheduler
    // with nothing to issue issued nothing, so its warps' head instructions
    // and scoreboards are unchanged; only flags (step 3's barriers, exits)
    // are read again
    const uint64_t valid_m = P::ballot_m(live, [&](int w) -> bool {
      const uint8_t f = s.w_flags[w];
      return (f & WF_ACTIVE) && !(f & (WF_EXITING | WF_BARRIER | WF_MEMBAR | WF_WAITCNT)) && s.w_ibuf[w] != 0 &&
             warp_issue_due(s, c, w, now);
    });
    const uint64_t sbok_m = valid_m & sbok_all;
    uint32_t n_c0 = 0, n_c1 = 0, n_c2 = 0;
    for (uint32_t sc = 0; sc < nsched; ++sc) {
      if (!(idle_sc >> sc & 1u)) continue;
      const uint32_t k = stall_class(c.sched_mask[sc], valid_m, sbok_m);
      n_c0 += k == 0;
      n_c1 += k == 1;
      n_c2 += k == 2;
    }
    s.sadd(SK(issue_stall_idle), n_idle);
    if (n_c0) s.sadd(SK(issue_distro) + 0, n_c0);
    if (n_c1) s.sadd(SK(issue_distro) + 1, n_c1);
    if (n_c2) s.sadd(SK(issue_distro) + 2, n_c2);
    P::prof(52);
  };
  if (!picks) {
    if (!classified) classify();
    return;
  }
  P::prof(50);
  s.last_progress = now;
  s.sadd(SK(busy_cycles), 1);
  const uint64_t spec = P::ballot_m(picks, [&](int w) -> bool { return issue_special(head.self(w)); });
  // 1. the pipeline issues in scheduler order, wave-uniform: statistics, ages,
  //    ID_OC registers (state that the per-warp step below does not touch)
  uint32_t age = P::uni(s.age_ctr);
  uint64_t idoc = P::uni(s.idoc_mask);
  for (uint32_t sc = 0; sc < nsched; ++sc) {
    const uint32_t w = (pk_of >> (8 * sc)) & 0xffu;
    if (w == 0xffu) continue;
    const TInst in = head.at((int)w);
    SADD_IN(s, issue_distro, 3 + kMaxWarpLanes, 2u + (uint32_t)amin<int>(popc64(in.mask), kMaxWarpLanes), 1);
    SADD_IN(s, single_issue, kMaxSched, sc, 1);
    if (spec >> w & 1ull) continue;  // step 3
    s.sadd(SK(warp_insn), 1);
    s.sadd(SK(thread_insn), (uint64_t)popc64(in.mask));
    SADD_IN(s, cls_insn, OC_COUNT, in.cls < OC_COUNT ? in.cls : OC_ALU, 1);
    SADD_IN(s, sq_insn, 8, sq_class(in), 1);
    if (in.space == S_CONST) s.sadd(SK(power_acc) + PWR_CONST_OPERAND, 1);
    {
      const uint32_t pk = (uint32_t)(in.flags >> 4);
      if (pk) SADD_IN(s, power_acc, 16, pk, pk == PWR_SALU ? 1ull : (uint64_t)popc64(in.mask));
    }
    const uint32_t u = unit_of(c, in.cls);
    const uint32_t kk = sc * U_COUNT + u;
    TInst ri = in;
    uint32_t lslot = 0xff;
    if (in.cls == OC_LOAD) {
      lslot = (uint32_t)ffs64((uint64_t)(uint8_t)~P::uni((uint8_t)s.w_slot_used[w]));
      if (in.space != S_SHARED && in.width == 0) {
        ri.space = S_SHARED;
        ri.width = 1;
      }
    } else if (in.cls == OC_STORE && in.space != S_SHARED && in.width == 0) {
      ri.space = S_SHARED;
      ri.width = 1;
    }
    s.idoc_inst[kk] = ri;
    s.idoc_meta[kk] = idoc_pack(w, lslot, ++age);
    idoc |= 1ull << kk;
  }
  s.age_ctr = age;
  s.idoc_mask = idoc;
  // 2. every pipeline-issuing warp's own state, one lane per warp
  P::prof(51);
  P::each_m(picks & ~spec, [&](int w) {
    const TInst in = head.self(w);
    s.w_head[w] = s.w_head[w] + 1u;
    s.w_ibuf[w] = (uint8_t)(s.w_ibuf[w] - 1u);
    s.w_inflight[w] = (uint8_t)(s.w_inflight[w] + 1u);
    const bool nomem = in.space != S_SHARED && in.width == 0;  // completes via the ring as an LDS op
    if (in.cls == OC_LOAD) {
      const uint8_t used = s.w_slot_used[w];
      const uint32_t sl = (uint32_t)ffs64((uint64_t)(uint8_t)~used);
      s.w_slot_used[w] = (uint8_t)(used | (1u << sl));
      s.w_loads[w] = (uint16_t)(s.w_loads[w] + 1u);
      uint32_t nacc = (in.space == S_SHARED) ? 1u : (uint32_t)in.width;
      if (nacc == 0) nacc = 1;
      s.w_slot_pend[w][sl] = (uint16_t)nacc;
      s.w_slot_dst[w][sl][0] = in.dst[0];
      s.w_slot_dst[w][sl][1] = in.dst[1];
      if (nomem || in.space == S_SHARED || in.space == S_CONST) s.w_slot_lds[w] = (uint8_t)(s.w_slot_lds[w] | (1u << sl));
    } else if (in.cls == OC_STORE && (nomem || in.space == S_SHARED)) {
      s.w_lds_st[w] = (uint8_t)(s.w_lds_st[w] + 1u);
    }
    sbs(s.w_sb, (uint32_t)w, in.dst[0]);
    sbs(s.w_sb, (uint32_t)w, in.dst[1]);
  });
  P::sync();
  P::prof(52);
  // 3. the instructions handled at issue, in scheduler order (the idle
  //    schedulers classified at the first of them)
  if (spec) {
    for (uint32_t sc = 0; sc < nsched; ++sc) {
      const uint32_t w = (pk_of >> (8 * sc)) & 0xffu;
      if (w == 0xffu || !(spec >> w & 1ull)) continue;
      if (!classified && sc > first_idle) classify();
      sm_issue_one<P>(s, x, now, sc, w, head.at((int)w), P::uni((uint32_t)s.w_head[w]));
    }
  }
  if (!classified) classify();
}

template <class P, class S>
SIM_HDI void sm_issue(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  const KernelTab& kt = *x.kt;
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const uint32_t nsched = c.n_sched ? c.n_sched : 1;
  const uint64_t idoc_busy = P::uni(s.idoc_mask);
  // every warp's next instruction, read once (a register per lane on the GPU)
  // (read straight from the kernel's trace in HBM: an L2-resident stream)
  P::fetch_wait();  // window entries DMA'd by earlier fetches
  const auto head = P::template lanes<TInst>(nw, [&](int w) -> TInst { return s.w_win[w][s.w_head[w] & (kWin - 1)]; });
  // readiness of every warp (lane-parallel)
  const uint64_t live = P::uni(s.live_mask);
  if ((c.sched_policy == SCHED_LRR || c.sched_policy == SCHED_GTO || c.sched_policy == SCHED_OLDEST ||
       c.sched_policy == SCHED_RRR) &&
      c.max_issue_per_warp <= 1 && !trace_sm_on(c, TS_WARP_SCHEDULER, s.id)) {
    // scoreboard and the rest of readiness as two masks: the stall
    // classification reuses the first
    const uint64_t sbok = P::ballot_m(live, [&](int w) -> bool { return warp_sb_ok(s, w, head.self(w)); });
    const uint64_t ready = P::ballot_m(live & sbok, [&](int w) -> bool {
      return warp_can_issue_nosb(s, c, w, head.self(w), nsched, idoc_busy) && warp_issue_due(s, c, w, now);
    });
    P::prof(29);
    sm_issue_par<P>(s, x, now, head, ready, live, sbok);
    return;
  }
  uint64_t ready = P::ballot_m(live, [&](int w) -> bool {
    return warp_can_issue_i(s, c, w, head.self(w), nsched, idoc_busy) && warp_issue_due(s, c, w, now);
  });
  // warps parked at a barrier / fence / exit (the reference's waiting()),
  // plus for the two-level scheduler those whose next instruction waits on
  // a long (memory) operation
  uint64_t waiting = 0;
  if (c.sched_policy == SCHED_WARP_LIMITING || c.sched_policy == SCHED_TWO_LEVEL)
    waiting = P::ballot_m(live, [&](int w) -> bool {
      const uint8_t f = s.w_flags[w];
      if (f & (WF_EXITING | WF_BARRIER | WF_MEMBAR | WF_WAITCNT)) return true;
      return c.sched_policy == SCHED_TWO_LEVEL && s.w_ibuf[w] && waits_long_op(s, w, head.self(w));
    });
  P::prof(29);
  bool issued_any = false;
  // issue-stall classification for the warp occupancy distribution, computed
  // only when a scheduler with live warps has nothing to issue
  uint64_t valid_m = 0, sbok_m = 0;
  bool classified = false;
  auto classify = [&]() {
    if (classified) return;
    classified = true;
    sm_stall_masks<P>(s, c, now, live, valid_m, sbok_m);
  };
  for (uint32_t sc = 0; sc < nsched; ++sc) {
    // warps of this scheduler
    const uint64_t mine = c.sched_mask[sc];
    uint64_t cand = ready & mine;
    const uint32_t last = P::uni((uint32_t)s.sched_last[sc]);
    if (c.sched_policy == SCHED_WARP_LIMITING && cand) {
      // swl_scheduler::order_warps (shader.cc:1686-1700): only the
      // sched_param oldest non-waiting warps (and the greedy one) compete
      uint64_t pool = live & mine & ~waiting, lim = 0;
      for (uint32_t i = 0; i < c.sched_param && pool; ++i) {
        const int o = P::argmin(nw, [&](int w) -> uint64_t {
          return (pool >> w & 1ull) ? ((uint64_t)s.w_age[w] << 8 | (uint64_t)w) : ~0ull;
        });
        if (o < 0) break;
        lim |= 1ull << o;
        pool &= ~(1ull << o);
      }
      if (last < (uint32_t)nw) lim |= 1ull << last;
      cand &= lim;
    } else if (c.sched_policy == SCHED_TWO_LEVEL && cand) {
      // two_level_active_scheduler (shader.cc:1599-1660): warps waiting on
      // long operations are demoted; the active set holds at most
      // sched_param warps, refilled in warp order; LRR inside it
      uint64_t pool = live & mine & ~waiting, act = 0;
      for (uint32_t i = 0; i < c.sched_param && pool; ++i) {
        const uint64_t b = pool & (~pool + 1);
        act |= b;
        pool &= ~b;
      }
      cand &= act;
    }
    if (!cand) {
      if (live & mine) {
        s.sadd(SK(issue_stall_idle), 1);
        classify();
        SADD_IN(s, issue_distro, 3 + kMaxWarpLanes, stall_class(mine, valid_m, sbok_m), 1);
      }
      continue;
    }
    int pick = -1;
    P::prof(43);
    switch (c.sched_policy) {
      case SCHED_GTO:
      case SCHED_WARP_LIMITING:
        if (last < (uint32_t)nw && (cand >> last & 1ull)) { pick = (int)last; break; }
        [[fallthrough]];
      case SCHED_OLDEST:
        pick = P::argmin(nw, [&](int w) -> uint64_t {
          return (cand >> w & 1ull) ? ((uint64_t)s.w_age[w] << 8 | (uint64_t)w) : ~0ull;
        });
        break;
      case SCHED_RRR: {
        uint32_t start = (uint32_t)(now % (uint64_t)nw);
        uint64_t r = rotr64(cand, start, (unsigned)nw);
        pick = (int)mod_small((uint32_t)ffs64(r) + start, (uint32_t)nw);
        break;
      }
      default: {  // LRR (and the two-level inner level): first ready warp after the last issued one
        uint32_t start = mod_small(last + 1, (uint32_t)nw);
        uint64_t r = rotr64(cand, start, (unsigned)nw);
        pick = (int)mod_small((uint32_t)ffs64(r) + start, (uint32_t)nw);
        break;
      }
    }
    P::prof(29);
    const uint32_t w = P::uni((uint32_t)pick);
    s.sched_last[sc] = w;
    if (c.warp_issue_interval > 1) P::one([&] { s.w_issue_ok[w] = now + c.warp_issue_interval; });
    const uint32_t hidx = P::uni((uint32_t)s.w_head[w]);
    const TInst in1 = head.at((int)w);
    P::prof(42);
    const int u1 = sm_issue_one<P>(s, x, now, sc, w, in1, hidx);
    P::prof(29);
    issued_any = true;
    SADD_IN(s, issue_distro, 3 + kMaxWarpLanes, 2u + (uint32_t)amin<int>(popc64(in1.mask), kMaxWarpLanes), 1);
    bool dual = false;
    // dual issue (reference scheduler_unit::cycle, shader.cc:1249-1556): the
    // warp's next buffered instruction issues in the same cycle if it is
    // ready and, with -gpgpu_dual_issue_diff_exec_units, uses another unit
    if (c.max_issue_per_warp > 1 && u1 >= 0 && P::uni((uint8_t)s.w_ibuf[w])) {
      const TInst in2 = P::uni(s.w_win[w][(hidx + 1) & (kWin - 1)]);  // the warp's next buffered instruction
      const bool special = in2.cls == OC_EXIT || in2.cls == OC_BARRIER || in2.cls == OC_MEMBAR ||
                           in2.cls == OC_NOP || (in2.flags & F_WAITCNT);
      if (!special && (!c.dual_issue_diff || unit_of(c, in2.cls) != (uint32_t)u1) &&
          warp_can_issue_i(s, c, (int)w, in2, nsched, P::uni(s.idoc_mask))) {
        sm_issue_one<P>(s, x, now, sc, w, in2, hidx + 1);
        s.sadd(SK(dual_issued), 1);
        SADD_IN(s, issue_distro, 3 + kMaxWarpLanes, 2u + (uint32_t)amin<int>(popc64(in2.mask), kMaxWarpLanes), 1);
        dual = true;
      }
    }
    if (dual) SADD_IN(s, dual_issue, kMaxSched, sc, 1);
    else SADD_IN(s, single_issue, kMaxSched, sc, 1);
  }
  if (issued_any) s.sadd(SK(busy_cycles), 1);
}

// ---------------------------------------------------------------------------
// fetch/decode: refill the instruction buffer of up to fetch_throughput
// warps whose buffer is empty (round-robin), perfect instruction cache
template <class P, class S>
SIM_HDI void sm_fetch(S& s, const SimCfg& c, const KernelTab& kt) {
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  P::fetch_wait();
  uint64_t need = P::ballot_m(P::uni(s.live_mask), [&](int w) {
    uint8_t f = s.w_flags[w];
    return (f & WF_ACTIVE) && !(f & (WF_EXITING | WF_IMISS)) && s.w_ibuf[w] == 0 && s.w_next[w] < s.w_end[w];
  });
  uint32_t start = mod_small(P::uni(s.fetch_rr), (uint32_t)nw);
  uint64_t r = rotr64(need, start, (unsigned)nw);
  const bool icache = !c.perfect_icache && !c.il1.disabled;
  for (uint32_t i = 0; i < c.fetch_throughput && r; ++i) {
    int b = ffs64(r);
    r &= r - 1;
    uint32_t w = mod_small((uint32_t)b + start, (uint32_t)nw);
    if (icache && !il1_fetch<P>(s, c, kt, w)) {
      s.fetch_rr = w + 1;  // miss / reservation fail ends this cycle's fetch (shader.cc:997-1010)
      break;
    }
    const uint32_t wnext = P::uni((uint32_t)s.w_next[w]);
    const uint32_t wend = P::uni((uint32_t)s.w_end[w]);
    uint32_t avail = wend - wnext;
    uint32_t n = avail < (uint32_t)kIbuf ? avail : (uint32_t)kIbuf;
    // window: [wnext] is already there (launch / previous fetch); bring in the
    // rest of this fetch and the next fetch's target
    for (uint32_t j = 1; j <= n && wnext + j < wend; ++j)
      P::fetch_copy(&s.w_win[w][(wnext + j) & (kWin - 1)], &inst_at(kt, wnext + j), 1);
    s.w_next[w] = wnext + n;
    s.w_ibuf[w] = (uint8_t)n;
    s.fetch_rr = w + 1;
  }
}

#if !defined(__HIP_DEVICE_COMPILE__)
[[noreturn]] inline void throw_cta_fit_error(uint32_t sm, uint32_t cta) {
  char b[128];
  snprintf(b, sizeof(b), "SM %u: no contiguous warp run for CTA %u (dispatch plan out of date)", sm, cta);
  throw std::logic_error(b);
}
#endif

// first warp of a free contiguous run of n warps among the first nw, or -1
// (shader_core_ctx::find_available_hwtid: a CTA's hardware threads are contiguous)
SIM_HDI int warp_run_fit(uint64_t used, uint32_t n, uint32_t nw) {
  if (n == 0 || n > nw) return -1;
  const uint64_t need = n >= 64 ? ~0ull : ((1ull << n) - 1);
  for (uint32_t b = 0; b + n <= nw; ++b)
    if (!((used >> b) & need)) return (int)b;
  return -1;
}

// resources a resident CTA gives back when it completes
template <class S>
SIM_HDI void sm_cta_release(S& s, const KernelTab& kt, uint32_t cta) {
  const uint32_t ks = s.cta_ks[cta];
  const KernelDesc& k = kt.k[ks];
  const uint32_t nw = s.cta_nw[cta];
  s.cta_wmask = s.cta_wmask & ~((nw >= 64 ? ~0ull : ((1ull << nw) - 1)) << s.cta_wbase[cta]);
  s.n_cta_k[ks] = (uint8_t)(s.n_cta_k[ks] - 1);
  s.used_thr = s.used_thr - k.thr_cta;
  s.used_regs = s.used_regs - k.regs_cta;
  s.used_shmem = s.used_shmem - k.shmem_per_cta;
}

// stream exhausted without explicit EXIT -> treat as exit
// warp retirement and CTA completion
template <class P, class S>
SIM_HDI void sm_retire(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const uint64_t live = P::uni(s.live_mask);
  uint64_t done = P::ballot_m(live, [&](int w) {
    uint8_t f = s.w_flags[w];
    if (!(f & WF_ACTIVE)) return false;
    bool drained = s.w_head[w] >= s.w_end[w] && s.w_ibuf[w] == 0;
    return drained && s.w_inflight[w] == 0 && s.w_stores[w] == 0 && s.w_loads[w] == 0;
  });
  // release membar / waitcnt waits
  if (P::uni(s.n_wait_flags)) {
    uint32_t released = 0;
    const uint64_t rel = P::ballot_m(live, [&](int w) {
      uint8_t f = s.w_flags[w];
      uint32_t r = 0;
      if ((f & WF_MEMBAR) && s.w_stores[w] == 0) { f = f & (uint8_t)~WF_MEMBAR; ++r; }
      if ((f & WF_WAITCNT) && waitcnt_met(s, w)) { f = f & (uint8_t)~WF_WAITCNT; ++r; }
      if (r) s.w_flags[w] = f;
      return r != 0;
    });
    // a warp waits on at most one of the two flags at a time
    released = (uint32_t)popc64(rel);
    s.n_wait_flags = P::uni(s.n_wait_flags) - released;
    P::sync();
  }
  while (done) {
    int w = ffs64(done);
    done &= done - 1;
    uint32_t cta = s.w_cta[w];
    if (!(s.w_flags[w] & WF_EXITING)) s.cta_nexit[cta]++;  // implicit exit at stream end
    s.w_flags[w] = 0;
    s.live_mask &= ~(1ull << w);
    s.n_warps_live--;
    s.sadd(SK(warps_done), 1);
    s.cta_live[cta]--;
    s.cta_nexit[cta]--;
    if (s.cta_live[cta] == 0) {
      s.cta_valid[cta] = 0;
      s.n_cta_active--;
      sm_cta_release(s, *x.kt, cta);
      s.sadd(SK(ctas_done), 1);
    } else {
      sm_barrier_check<P>(s, cta);
    }
    s.last_progress = now;
  }
}

// ---------------------------------------------------------------------------
// launch CTA `cta_id` of the kernel in slot `ks` into CTA slot `slot`, on the
// first contiguous run of free warps
template <class P, class S>
SIM_HDI void sm_launch_cta(S& s, const SmCtx& x, uint32_t slot, uint32_t cta_id, uint32_t ks) {
  const KernelDesc& k = x.kt->k[ks];
  const SimCfg& c = *x.cfg;
  const uint32_t wpc = k.warps_per_cta;
  const uint32_t nwm = amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const int fit = warp_run_fit(s.cta_wmask, wpc, nwm);  // planned by sm_cta_fit at the last boundary
  if (fit < 0) {
    // the plan no longer matches the SM (cannot happen while the kernel table
    // and the SM state evolve together); never index warps with -1
#if !defined(__HIP_DEVICE_COMPILE__)
    throw_cta_fit_error(s.id, cta_id);
#endif
    return;
  }
  const uint32_t base = (uint32_t)fit;
  const uint64_t wm = (wpc >= 64 ? ~0ull : ((1ull << wpc) - 1)) << base;
  if (s.n_cta_active == 0) {
    // an empty SM takes the kernel's L1 / shared-memory carve-out
    s.l1_sets = (uint16_t)k.l1_sets;
    s.l1_assoc = (uint16_t)k.l1_assoc;
  }
  s.cta_valid[slot] = 1;
  s.cta_id[slot] = cta_id;
  s.cta_live[slot] = (uint8_t)wpc;
  s.cta_bar[slot] = 0;
  s.cta_nexit[slot] = 0;
  s.cta_ks[slot] = (uint8_t)ks;
  s.cta_wbase[slot] = (uint8_t)base;
  s.cta_nw[slot] = (uint8_t)wpc;
  s.cta_wmask |= wm;
  s.n_cta_k[ks]++;
  s.used_thr += k.thr_cta;
  s.used_regs += k.regs_cta;
  s.used_shmem += k.shmem_per_cta;
  s.n_cta_active++;
  s.n_warps_live += wpc;
  s.live_mask |= wm;
  uint32_t age0 = s.age_ctr;
  s.age_ctr += wpc;
  const uint32_t tag = ks << kSlotShift;
  P::each((int)wpc, [&](int i) {
    uint32_t w = base + (uint32_t)i;
    WStream ws = k.streams[(uint64_t)(cta_id & k.cmask) * wpc + (uint32_t)i];
    s.w_next[w] = tag | ws.begin;
    s.w_head[w] = tag | ws.begin;
    s.w_end[w] = tag | (ws.begin + ws.count);
    if (ws.count) s.w_win[w][ws.begin & (kWin - 1)] = k.insts[ws.begin & k.imask];  // the first fetch's target
    s.w_issue_ok[w] = 0;
    s.w_age[w] = age0 + (uint32_t)i;
    s.w_flags[w] = WF_ACTIVE;
    s.w_iline[w] = 0;  // no code block fetched yet
    s.w_ibuf[w] = 0;
    s.w_cta[w] = (uint8_t)slot;
    s.w_inflight[w] = 0;
    s.w_stores[w] = 0;
    s.w_loads[w] = 0;
    s.w_slot_used[w] = 0;
    s.w_slot_lds[w] = 0;
    s.w_lds_st[w] = 0;
    s.w_wait[w] = 0;
    sbz(s.w_sb, w);
  });
  P::sync();
}

// one simulated core cycle
template <class P, class S>
SIM_HDI void sm_cycle(S& s, const SmCtx& x, uint64_t now) {
  const SimCfg& c = *x.cfg;
  P::prof(0);
  sm_receive<P>(s, x, now);
  P::prof(1);
  sm_writeback<P>(s, c, now);
  P::prof(2);
  sm_hit_complete<P>(s, now);
  P::prof(3);
  sm_ldst<P>(s, x, now);
  P::prof(4);
  sm_dispatch<P>(s, x, now);
  P::prof(5);
  sm_read_operands<P>(s, c);
  P::prof(6);
  sm_alloc_collectors<P>(s, c);
  P::prof(7);
  sm_issue<P>(s, x, now);
  P::prof(8);
  sm_fetch<P>(s, c, *x.kt);
  P::prof(9);
  sm_retire<P>(s, x, now);
  P::prof(10);
  sm_inject<P>(s, x, now);
  P::prof(11);
  if (P::uni(s.n_cta_active)) {
    s.sadd(SK(active_cycles), 1);
    s.sadd(SK(occupancy_acc), P::uni(s.n_warps_live));
  }
}

// true if the SM holds no work at all (no CTAs, nothing in flight)
template <class S>
SIM_HDI bool sm_idle(const S& s) {
  return s.n_cta_active == 0 && s.outq_n == 0 && s.outstanding == 0 && !s.ldst.busy && s.cl_n == 0 && s.ld_n == 0;
}

// first cycle in [from, limit) whose slot of a time-indexed ring is occupied:
// the occupied slot at the smallest circular distance from `from` (one
// candidate per 64-slot word, lane-parallel; the GPU view keeps the words in
// registers)
template <class P, class A>
SIM_HDI uint64_t ring_next(const A& occ, uint32_t ring, uint64_t from, uint64_t limit) {
  const uint32_t nwords = ring / 64;
  const uint32_t start = (uint32_t)(from % ring);
  const uint32_t w0 = start >> 6, b0 = start & 63;
  auto dist = [&](int i) -> uint64_t {
    const uint64_t m = occ[i];
    if (!m) return ~0ull;
    const uint64_t mh = (uint32_t)i == w0 ? (m & (~0ull << b0)) : m;
    const uint32_t p = (uint32_t)i * 64u + (uint32_t)ffs64(mh ? mh : m);
    return (uint64_t)((p + ring - start) & (ring - 1));
  };
  const int j = P::argmin((int)nwords, dist);
  if (j < 0) return limit;
  return amin<uint64_t>(limit, from + P::uni(dist(j)));
}

// Exact quiescence test before simulating cycle `t`: if no stage of
// sm_cycle can change state until some later cycle, return that cycle
// (capped at `limit`); otherwise return `t`.  Quiet cycles only add the
// per-cycle statistics (sm_skip).  This is what makes latency-bound phases
// (every warp waiting on memory) cost one check instead of one cycle each.
template <class P, class S>
SIM_HDI uint64_t sm_quiet_until(const S& s, const SimCfg& c, const KernelTab& kt, uint64_t t, uint64_t limit) {
  if (P::uni(s.ldst.busy) || P::uni(s.idoc_mask) || P::uni(s.oc_mask | s.oc_read_mask) || P::uni(s.outq_n) ||
      P::uni(s.cl_n | s.ld_n))
    return t;
  uint64_t nx = ring_next<P>(s.wb_occ, kWbRing, t, limit);
  if (nx == t) return t;
  nx = ring_next<P>(s.hit_occ, kHitRing, t, nx);
  if (nx == t) return t;
  if (P::uni(s.inq_n)) {
    const uint64_t at = core_cyc_ceil(c, P::uni(s.inq[P::uni(s.inq_head)].t));
    if (at <= t) return t;
    nx = amin<uint64_t>(nx, at);
  }
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const uint32_t nsched = c.n_sched ? c.n_sched : 1;
  const uint64_t act = P::ballot_m(P::uni(s.live_mask), [&](int w) -> bool {
    const uint8_t f = s.w_flags[w];
    if (!(f & WF_ACTIVE)) return false;
    if (!(f & (WF_EXITING | WF_IMISS)) && s.w_ibuf[w] == 0 && s.w_next[w] < s.w_end[w]) return true;  // fetch
    const bool drained = s.w_head[w] >= s.w_end[w] && s.w_ibuf[w] == 0;
    if (drained && s.w_inflight[w] == 0 && s.w_stores[w] == 0 && s.w_loads[w] == 0) return true;  // retire
    if ((f & WF_MEMBAR) && s.w_stores[w] == 0) return true;
    if ((f & WF_WAITCNT) && waitcnt_met(s, w)) return true;
    return warp_can_issue(s, c, kt, w, nsched, s.idoc_mask) && warp_issue_due(s, c, w, t);  // issue
  });
  if (act) return t;
  if (c.warp_issue_interval > 1) {
    // warps held only by their issue interval wake when it ends
    const int o = P::argmin(nw, [&](int w) -> uint64_t {
      if (!(P::uni(s.live_mask) >> w & 1ull)) return ~0ull;
      return warp_can_issue(s, c, kt, w, nsched, s.idoc_mask) && !warp_issue_due(s, c, w, t) ? s.w_issue_ok[w]
                                                                                                : ~0ull;
    });
    if (o >= 0) nx = amin<uint64_t>(nx, P::uni((uint64_t)s.w_issue_ok[o]));
  }
  return nx;
}

// account `k` quiet cycles: exactly what k idle sm_cycle calls would add
template <class P, class S>
SIM_HDI void sm_skip(S& s, const SimCfg& c, uint64_t k, uint64_t t) {
  const int nw = (int)amin<uint32_t>(c.max_warps_per_sm, kMaxWarps);
  const uint32_t nsched = c.n_sched ? c.n_sched : 1;
  const uint64_t live = P::uni(s.live_mask);
  uint32_t stalled = 0;
  uint64_t valid_m = 0, sbok_m = 0;
  if (live) sm_stall_masks<P>(s, c, t, live, valid_m, sbok_m);  // constant over the quiet cycles
  for (uint32_t sc = 0; sc < nsched; ++sc) {
    if (live & c.sched_mask[sc]) {
      ++stalled;
      SADD_IN(s, issue_distro, 3 + kMaxWarpLanes, stall_class(c.sched_mask[sc], valid_m, sbok_m), k);
    }
  }
  // uniform update by every lane (not P::one: on the GPU these fields may be
  // registers of a view, which a one-lane write would leave divergent)
  s.sadd(SK(issue_stall_idle), (uint64_t)stalled * k);
  if (P::uni(s.n_cta_active)) {
    s.sadd(SK(active_cycles), k);
    s.sadd(SK(occupancy_acc), (uint64_t)popc64(live) * k);
  }
  s.skipped_cycles += k;
  P::sync();
}

}  // namespace asim
