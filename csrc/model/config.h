// POD configuration consumed by the cycle model (host AND device).
//
// Produced on the host from the gpgpusim.config / trace.config option
// registry (csrc/config/sim_options.cc) -- the reference spreads the same
// information over gpgpu_sim_config / shader_core_config / memory_config
// (gpu-sim.h:97-473, shader.h:1509-1716).  Copied once to device memory.
#pragma once
#include "types.h"

namespace asim {

// compile-time capacity caps of the fixed-size state (checked by the host
// when a config is loaded; configs beyond them are rejected loudly)
constexpr int kMaxWarps = 64;       // warps per SM (lanes of one wavefront)
constexpr int kMaxWarpLanes = 64;   // threads per warp (wave64)
constexpr int kMaxCta = 32;         // CTA slots per SM
constexpr int kMaxSched = 4;        // schedulers / sub-cores per SM
constexpr int kIbuf = 2;            // instruction buffer entries per warp
constexpr int kWin = 4;             // per-warp decoded-instruction window [w_head, w_next] (>= kIbuf + 1, power of 2)
constexpr int kMaxEpoch = 256;     // longest PDES epoch (interconnect lookahead), core cycles
constexpr int kMaxOC = 16;          // operand collector units per SM
constexpr int kMaxBanks = 32;       // register file banks per SM
constexpr int kWbRing = 512;        // writeback ring (max FU latency 511)
constexpr int kWbSlot = 8;          // writebacks per cycle (EX_WB width cap)
constexpr int kMaxL1Lines = 1024;   // 128 KB of 128 B lines
constexpr int kMaxL1Mshr = 256;
constexpr int kMaxIL1Lines = 512;  // instruction cache: 64 KB of 128 B lines
constexpr int kMaxIL1Mshr = 16;
constexpr int kMaxCL1Lines = 1024; // constant / scalar data cache: 64 KB of 64 B lines
constexpr int kMaxCL1Mshr = 32;
constexpr uint64_t kProgramMemStart = 0xF0000000ull;  // code address base (reference PROGRAM_MEM_START)
constexpr uint64_t kScalarBase = 0x7FFE00000000ull;   // data addresses keyed to CDNA scalar loads (coalesce_kernel)
constexpr int kMaxPend = 1024;      // outstanding (warp,load-slot,line) L1 waiters
constexpr int kLoadSlots = 8;       // in-flight load instructions per warp
constexpr int kHitRing = 256;       // L1 / shared-memory completion ring (latency < 222)
constexpr int kHitSlot = 8;
constexpr int kOutQ = 64;           // SM -> icnt injection queue
constexpr int kInQ = 128;           // icnt -> SM arrivals per epoch
constexpr int kEjectQ = 32;         // cluster ejection buffer (-gpgpu_n_cluster_ejection_buffer_size cap)
constexpr int kLdstRespQ = 8;       // LD/ST response FIFO (-gpgpu_n_ldst_response_buffer_size cap)
constexpr int kMaxAccess = 64;      // coalesced accesses of one instruction
// memory side (per sub-partition)
constexpr int kMaxXcd = 16;        // XCDs (-sim_xcd)
constexpr int kMaxL2LinesCh = 2048; // per memory channel, shared by its sub-partitions
constexpr int kMaxL2Mshr = 256;
constexpr int kMaxL2Wait = 256;
constexpr int kRopQ = 256;
constexpr int kMemInQ = 256;        // arrivals per epoch per sub-partition
constexpr int kReplyQ = 128;
constexpr int kDramQ = 128;         // per channel FR-FCFS queue
constexpr int kDramLat = 512;       // per channel L2->DRAM latency pipe (in flight >= dram_latency x 1/cycle)
constexpr int kDramRet = 256;
constexpr int kMallRet = 64;        // MALL read hits waiting to return to the L2 (per channel)
constexpr int kMaxBanksDram = 32;
constexpr int kMaxSubPerCh = 2;
constexpr int kMaxSubTot = 128;    // L2 sub-partitions (interconnect destinations)
constexpr int kMaxSmTot = 512;     // simulated SMs

enum SchedPolicy : uint8_t { SCHED_LRR = 0, SCHED_GTO, SCHED_OLDEST, SCHED_RRR, SCHED_TWO_LEVEL, SCHED_WARP_LIMITING };
enum ReplPolicy : uint8_t { REPL_LRU = 0, REPL_FIFO };
enum WritePolicy : uint8_t { WP_READ_ONLY = 0, WP_WRITE_BACK, WP_WRITE_THROUGH, WP_WRITE_EVICT, WP_LOCAL_WB_GLOBAL_WT };
enum SetIndexFn : uint8_t { SIDX_LINEAR = 0, SIDX_FERMI, SIDX_HASH_IPOLY, SIDX_BITWISE_XOR, SIDX_CUSTOM };
enum PartIndex : uint8_t { PIDX_CONSECUTIVE = 0, PIDX_BITWISE = 1, PIDX_IPOLY = 2, PIDX_PAE = 3, PIDX_RANDOM = 4, PIDX_CUSTOM = 5 };
enum AddrField : uint8_t { AF_CHIP = 0, AF_BK, AF_ROW, AF_COL, AF_BURST, AF_COUNT };

// a bit-gather mask as contiguous runs: field = OR_i ((v >> sh[i]) & (2^w[i]-1)) << out[i]
// (n = 0xff: more than 8 runs, gather bit by bit)
struct BitRuns {
  uint8_t n;
  uint8_t sh[8];
  uint8_t w[8];
  uint8_t out[8];
  uint8_t pad[7];
};

struct CacheGeom {
  uint32_t nsets;
  uint32_t assoc;
  uint32_t line;        // bytes
  uint32_t mshr_entries;
  uint32_t mshr_merge;
  uint32_t miss_queue;
  uint8_t sectored;
  uint8_t repl;         // ReplPolicy
  uint8_t wpolicy;      // WritePolicy
  uint8_t alloc;        // 'm' on-miss 'f' on-fill 's' streaming
  uint8_t walloc;       // 'N' no-write-allocate, 'W' write-allocate, 'F' fetch-on-write, 'L' lazy
  uint8_t set_index;    // SetIndexFn
  uint8_t disabled;
  uint8_t pad;
};

// Debug trace streams (reference gem5-style DPRINTF streams, trace.h:28-92,
// trace_streams.tup: -trace_enabled / -trace_components / -trace_sampling_*).
// Units append fixed-size events to per-unit buffers; the host drains and
// prints them in (cycle, unit, order) order, identically for both engines.
enum TraceStream : uint32_t {
  TS_WARP_SCHEDULER = 1u << 0,
  TS_SCOREBOARD = 1u << 1,
  TS_MEMORY_PARTITION_UNIT = 1u << 2,
  TS_MEMORY_SUBPARTITION_UNIT = 1u << 3,
  TS_INTERCONNECT = 1u << 4,
  TS_LIVENESS = 1u << 5,
};
enum TraceKind : uint16_t {
  EV_ISSUE = 1,      // a = warp, b = pc | opcode << 32
  EV_SB_RELEASE,     // a = warp, b = register
  EV_PKT_SEND,       // a = destination sub-partition, b = line address
  EV_PKT_RECV,       // a = packet type, b = line address
  EV_L2_ACCESS,      // a = sub << 8 | outcome (0 hit, 1 miss, 2 mshr hit, 3 bypass/atomic), b = line
  EV_DRAM_CMD,       // a = command (0 RD, 1 WR, 2 ACT, 3 PRE), b = bank << 32 | row
};
struct TraceEv {
  uint64_t cycle;  // core cycle (SM events) or DRAM cycle (DRAM commands) / femtoseconds>>10 (L2)
  uint32_t unit;   // SM id, or n_sm + channel id
  uint16_t kind;
  uint16_t a;
  uint64_t b;
};

// Exact unsigned 64-bit division by a divisor fixed for the run (the clock
// periods): a multiply-high and a shift instead of the ~100-instruction
// software division the GPU would otherwise run for every `/ per_core`
// (round-up magic numbers, Granlund & Montgomery 1994; the same arithmetic
// on both engines, so results stay bit-identical).
struct Div64 {
  uint64_t magic;  // 0: power of two (shift only)
  uint64_t d;
  uint32_t shift;
  uint32_t add;    // the 65-bit magic's top bit: q = (((x - hi) >> 1) + hi) >> shift
};
SIM_HDI uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
SIM_HDI uint64_t fdiv(uint64_t x, const Div64& v) {
  if (!v.magic) return x >> v.shift;
  const uint64_t hi = mulhi64(x, v.magic);
  if (v.add) return (((x - hi) >> 1) + hi) >> v.shift;
  return hi >> v.shift;
}
// host only (called at config time; plain host functions are parsed, never
// emitted, in the device pass)
inline Div64 make_div64(uint64_t d) {
  Div64 r{0, d ? d : 1, 0, 0};
  d = r.d;
  const uint32_t l = 63u - (uint32_t)__builtin_clzll(d);  // floor(log2 d)
  if ((d & (d - 1)) == 0) {
    r.shift = l;
    return r;
  }
  // m = floor(2^(64+l) / d); the smallest power that works gives a 64-bit
  // magic, otherwise the 65-bit one with the add step
  const unsigned __int128 num = (unsigned __int128)1 << (64 + l);
  uint64_t m = (uint64_t)(num / d);
  const uint64_t rem = (uint64_t)(num % d);
  const uint64_t e = d - rem;
  if (e < (1ull << l)) {
    r.shift = l;
    r.add = 0;
  } else {
    m += m;
    const uint64_t twice = rem + rem;
    if (twice >= d || twice < rem) m += 1;
    r.shift = l;
    r.add = 1;
  }
  r.magic = m + 1;
  return r;
}

struct SimCfg {
  // ---- topology ----
  uint32_t n_sm;
  uint32_t n_clusters;
  uint32_t cores_per_cluster;
  uint32_t n_mem;           // DRAM channels
  uint32_t n_sub_per_mem;   // L2 sub-partitions per channel
  uint32_t n_subpart;       // n_mem * n_sub_per_mem
  uint32_t warp_size;       // threads per warp in the traces (32 SASS, 64 CDNA)
  // ---- SM resources ----
  uint32_t max_threads_per_sm;
  uint32_t max_warps_per_sm;
  uint32_t max_cta_per_sm;
  uint32_t regs_per_sm;
  uint32_t shmem_per_sm;
  uint32_t shmem_per_block;
  uint32_t concurrent_kernel_sm;  // -gpgpu_concurrent_kernel_sm: CTAs of several kernels share an SM
  uint32_t max_concurrent_kernel; // running kernels (<= kMaxConc)
  // ---- front end / issue ----
  uint32_t n_sched;
  uint32_t sched_policy;
  uint64_t sched_mask[kMaxSched];  // warps (lanes) supervised by each scheduler: w % n_sched == sc
  uint32_t sub_core;
  uint32_t fetch_throughput;
  uint32_t max_issue_per_warp;
  uint32_t warp_issue_interval;   // cycles between two issue cycles of one warp (CDNA: a wave issues once per SIMD visit)
  uint32_t dual_issue_diff;      // -gpgpu_dual_issue_diff_exec_units
  uint32_t sched_param;          // two_level_active:<max active>, warp_limiting:<prio>:<warps>
  // ---- execution ----
  uint32_t unit_count[U_COUNT];   // total units of each type per SM (0 = absent)
  uint32_t id_oc_width[U_COUNT];  // ID_OC pipeline register slots per type
  uint32_t ex_wb_width;
  uint16_t lat[OC_COUNT];         // latency per op class (trace mode)
  uint16_t ii[OC_COUNT];          // initiation interval per op class
  uint32_t oc_units;              // generic operand collector units per SM
  uint32_t reg_banks;
  uint32_t reg_port_tp;           // register file port throughput
  // ---- LD/ST ----
  uint32_t smem_banks;
  uint32_t smem_latency;
  uint32_t smem_warp_parts;
  uint32_t smem_limited_bcast;
  uint32_t smem_cdna_groups;  // wave64 LDS banking by the CDNA4 per-instruction lane groups (trace.cc lds_groups)
  uint32_t smem_pad_;
  CacheGeom l1;
  uint32_t l1_latency;
  // -sim_l1_miss_return_latency: cycles from a line's fill (or a bypassing
  // reply) to the waiting load's completion -- the vector memory pipeline a
  // miss traverses on CDNA besides the L2 round trip (0: none, GPGPU-Sim)
  uint32_t l1_miss_ret;
  uint32_t l1_banks;
  // L1 data path throughput (0 = off, the reference's banked L1: l1_banks
  // accesses per cycle): a global / local instruction occupies the vector
  // L1's address stage ceil(active lanes / l1_addr_lanes) cycles, each access
  // its data stage ceil(bytes / l1_port_bytes) cycles (gfx950 TA / TD)
  uint32_t l1_port_bytes, l1_addr_lanes;
  // -sim_l1_port_granule: the data stage moves whole 32 B sectors / 64 B
  // halves of a line (0: the bytes the lanes touch)
  uint32_t l1_port_granule;
  // LDS data path (0 = off: an LDS instruction takes its bank-conflict degree
  // in cycles): at least ceil(active lanes x bytes / lds_port_bytes) cycles,
  // computed at ingest into the instruction's initiation interval
  uint32_t lds_port_bytes, lds_lanes;  // lds_lanes: address lanes per cycle (0: no limit)
  uint32_t gmem_skip_l1;
  uint32_t adaptive_l1;
  uint32_t unified_l1_kb;
  uint32_t n_shmem_opts;
  uint32_t shmem_opts_kb[8];
  uint32_t l1_write_ratio;
  // ---- instruction cache (reference m_L1I read_only_cache, shader.cc:918-1020;
  //      -gpgpu_perfect_inst_const_cache bypasses it, shader.cc:990) ----
  CacheGeom il1;
  uint32_t perfect_icache;
  uint32_t inst_prefetch;   // L1I sequential prefetch depth in lines (CDNA SQC fetches ahead)
  uint32_t ifetch_block;    // > 0: a warp probes the L1I only when its fetch enters a new block of this many bytes
  uint32_t ifetch_pad_;
  // ---- constant cache (reference m_L1C read_only_cache, ldst_unit::
  //      constant_cycle, shader.cc:2196-2225, fills shader.cc:2819-2823); on
  //      CDNA the scalar data cache of the SQC that s_load reads through ----
  CacheGeom cl1;
  uint32_t cl1_latency;     // hit latency (core cycles); -sim_const_cache_latency, 0 = the L1D's
  uint32_t cl1_flush;       // invalidate it with the L1D at a kernel's start (the CDNA dispatch's acquire)
  // ---- interconnect ----
  uint32_t icnt_latency;   // core cycles (== epoch length, the PDES lookahead)
  uint32_t flit_size;
  // crossbar output-port arbitration (local_interconnect.cc:123-270):
  // 0 = round robin with a rotating global pointer, 1 = iSLIP (per-output
  // pointer advanced past the granted input every icnt_grant_cycles grants)
  uint32_t icnt_arbiter, icnt_grant_cycles;
  uint32_t icnt_in_pkts;  // SM injection buffer (-icnt_in_buffer_limit flits) in max-size packets
  uint32_t icnt_out_limit; // per-SM outstanding packets before injection stalls
  // reply path into the SM (reference simt_core_cluster::icnt_cycle and
  // ldst_unit::cycle, shader.cc:4623-4660, 2302-2309, 2810-2857): packets
  // leave the crossbar into the cluster's ejection buffer, move to the LD/ST
  // unit's response FIFO, and are consumed there one per cycle
  uint32_t eject_buf;      // -gpgpu_n_cluster_ejection_buffer_size (packets)
  uint32_t ldst_resp_buf;  // -gpgpu_n_ldst_response_buffer_size (packets)
  // -network_mode 1 (intersim2 / Booksim topologies, reference
  // icnt_wrapper.cc:35-45 + intersim2/networks/*): per-pair latency from the
  // topology's hop count and the router pipeline; icnt_latency above is then
  // the minimum over all SM<->sub-partition pairs (the PDES lookahead)
  uint32_t icnt_mode;       // 1 topology (intersim), 2 local crossbar (fixed latency)
  uint8_t topo;             // IcntTopo
  uint8_t topo_n;           // dimensions / stages / tree levels
  uint16_t topo_k;          // radix
  uint16_t topo_conc;       // nodes per router (cmesh concentration)
  uint16_t hop_icnt;        // icnt cycles per router traversal (routing + VA + SA + ST)
  uint16_t chan_icnt;       // icnt cycles per channel
  uint16_t link_contention;  // -icnt_link_contention: 1 link reservations (icnt_links.h), 2 input-queued routers (icnt_router.h)
  // input-queued router microarchitecture of -icnt_link_contention 2 (the
  // .icnt file's num_vcs, vc_buf_size, alloc_iters, credit_delay,
  // sw_allocator, sw_alloc_delay and internal_speedup)
  uint8_t rt_vcs, rt_iters, rt_credit, rt_alloc, rt_sa;
  uint8_t rt_route;        // routing_function: 0 deterministic (the topology's), 1 minimal adaptive (min_adapt), 2 Valiant
  uint16_t rt_buf;         // flits per virtual channel
  uint16_t rt_speedup_q8;  // switch passes per cycle x 256
  uint16_t rt_inbuf;       // input_buffer_size: flits a node's injection queue holds (HasBuffer)
  // ---- memory partition ----
  CacheGeom l2;
  uint32_t rop_latency;
  uint32_t dram_latency;
  uint32_t q_icnt_l2, q_l2_dram, q_dram_l2, q_l2_icnt;
  uint32_t perf_memcpy;
  // ---- DRAM ----
  uint32_t dram_sched;      // 0 FIFO, 1 FR-FCFS
  uint32_t dram_queue;
  uint32_t dram_ret_queue;
  uint32_t dram_credits;    // L2->DRAM in-flight limit per channel (latency pipe + scheduler queue)
  uint32_t nbk, nbkgrp, tCCD, tRRD, tRCD, tRAS, tRP, tRC, CL, WL, tCDLR, tWR, tCCDL, tRTPL;
  uint32_t BL, busW, data_cmd_ratio, dual_bus, bk_index_policy, bkgrp_index_policy;
  uint32_t atom_size;       // bytes per DRAM column access
  uint32_t rw_turnaround;   // 0: -dram_elimnate_rw_turnaround (tWTR = tRTW = 0)
  uint32_t wq_enable;       // -dram_seperate_write_queue_enable
  uint32_t wq_size, wq_hi, wq_lo;  // -dram_write_queue_size <size>:<high>:<low watermark>
  // ---- address decode ----
  uint64_t addr_mask[AF_COUNT];
  uint8_t mk_hi[AF_COUNT];
  uint8_t mk_lo[AF_COUNT];
  uint8_t part_index;
  uint8_t gap;
  int32_t addr_chip_s;
  uint32_t log2ch, log2sub, n_ch_pow2;
  uint64_t sub_id_mask;
  BitRuns addr_runs[AF_COUNT];  // addr_mask[f] restricted to [mk_lo, mk_hi), as runs
  BitRuns part_runs;            // partition_address gather mask as runs
  // ---- clocks (femtoseconds per cycle) ----
  uint64_t per_core, per_icnt, per_l2, per_dram;
  // core-clock time base: core cycle clk_base_cyc began at clk_base_fs, and
  // every later core cycle lasts per_core.  DVFS (-dvfs_enabled with a power
  // cap) changes per_core at an epoch boundary by moving the base there, so
  // the stamps already taken in femtoseconds stay valid (core_fs / core_cyc)
  uint64_t clk_base_cyc, clk_base_fs;
  uint64_t per_core_max;    // the longest core period DVFS may set (sizes the per-epoch reply mailboxes)
  Div64 dv_core, dv_icnt, dv_l2, dv_dram;  // exact division by the periods (cfg_set_divs)
  Div64 dv_epoch;                          // ... and by the epoch length (icnt_latency)
  // ---- kernel scheduling ----
  uint32_t kernel_launch_latency;
  uint32_t kernel_launch_latency_queued;  // a kernel right behind the previous one (driver)
  uint32_t tb_launch_latency;
  // ---- misc ----
  uint32_t deadlock_window;
  // run caps checked every epoch (-gpgpu_max_insn, -gpgpu_max_completed_cta)
  uint64_t max_insn;
  uint32_t max_completed_cta;
  // -gpu_trace_window W (GPU engine): keep only a window of about W x the
  // resident-CTA capacity of a kernel's trace in HBM, streamed in as CTAs
  // dispatch (0 = the whole kernel); the host engines ignore it
  uint32_t trace_window;
  uint32_t max_cycle_lo, max_cycle_hi;
  // ---- idealisations (reference -gpgpu_perfect_mem, perfect_memory_interface
  //      shader.h:2681; -gpgpu_simple_dram_model, l2cache.cc:235-303) ----
  uint32_t perfect_mem;     // every global/local access hits with L1 latency, no traffic
  uint32_t simple_dram;     // DRAM = latency pipe + one column per DRAM cycle, no bank timing
  uint32_t event_skip;      // fast-forward provably quiet SM cycles inside an epoch (exact)
  // ---- CDNA4 memory hierarchy (MI355X-native extension; 0 = the reference's
  //      single address-interleaved L2, l2cache.cc:463-595) ----
  // -sim_xcd N: the SMs form N XCDs (SM s -> XCD s % N, the workgroup
  // round-robin of the hardware dispatcher) with PRIVATE L2s: XCD x owns
  // sub-partitions [x*spx, (x+1)*spx), spx = n_subpart / N, and an SM's
  // request goes to the slice of its own XCD selected by the address.  Data
  // read by several XCDs is cached (and missed) in each of them.
  uint32_t n_xcd;
  uint32_t l1_wr_req_bytes;  // -sim_l1_write_request_bytes: 64 = a store is one request per 64 B half line
  // -sim_single_valu: CDNA issues every vector ALU instruction -- integer,
  // fp32, fp64, transcendental -- through the SIMD's one VALU (only MFMA has
  // its own matrix core): the INT / DP / SFU classes share the SP unit of
  // their scheduler, each at its own initiation interval, instead of running
  // in separate pipelines next to each other as on an NVIDIA sub-core
  uint32_t single_valu;
  uint32_t log2_spx;        // log2(sub-partitions per XCD)
  // -sim_mall <sets>:<assoc>: the memory-attached last-level cache (AMD
  // Infinity Cache / MALL) in front of every DRAM channel, sectored like the
  // L2, write-back; L2 misses that hit it return without a DRAM access, HBM
  // accesses pay -sim_mall_miss_latency on top of the DRAM timing
  uint32_t mall_sets, mall_assoc;
  uint64_t mall_miss_fs;    // extra latency of a MALL miss (fs)
  uint32_t cpu_threads;     // CPU engine only: OpenMP threads per epoch (host option)
  // ---- debug trace streams (pointers are set by the engine that owns the buffers) ----
  uint32_t trace_mask;      // TraceStream bits
  int32_t trace_sm;         // -trace_sampling_core (-1: all)
  int32_t trace_mem;        // -trace_sampling_memory_partition (-1: all)
  uint32_t trace_cap;       // events per unit per drain
  TraceEv* trace_ev;        // [units][trace_cap]
  uint32_t* trace_cnt;      // [units]
};

// append one event for `unit` (call from code that one lane executes, or all
// lanes redundantly through P::one)
SIM_HDI void trace_put(const SimCfg& c, uint32_t unit, uint64_t cycle, uint16_t kind, uint16_t a, uint64_t b) {
  uint32_t n = c.trace_cnt[unit];
  if (n < c.trace_cap) {
    TraceEv& e = c.trace_ev[(uint64_t)unit * c.trace_cap + n];
    e.cycle = cycle;
    e.unit = unit;
    e.kind = kind;
    e.a = a;
    e.b = b;
  }
  c.trace_cnt[unit] = n + 1;
}
enum IcntTopo : uint8_t { TOPO_FLY = 0, TOPO_MESH, TOPO_TORUS, TOPO_CMESH, TOPO_FATTREE, TOPO_FLATFLY };

// routers a packet traverses between interconnect nodes a and b
SIM_HDI uint32_t icnt_routers(const SimCfg& c, uint32_t a, uint32_t b) {
  const uint32_t k = c.topo_k ? c.topo_k : 2, n = c.topo_n ? c.topo_n : 1;
  switch (c.topo) {
    case TOPO_FLY:  // k-ary n-fly: every route crosses all n stages
      return n;
    case TOPO_CMESH:
      a /= (c.topo_conc ? c.topo_conc : 1);
      b /= (c.topo_conc ? c.topo_conc : 1);
      [[fallthrough]];
    case TOPO_MESH:
    case TOPO_TORUS: {  // k-ary n-cube, dimension-order routing
      uint32_t h = 0;
      for (uint32_t d = 0; d < n; ++d) {
        const uint32_t x = a % k, y = b % k;
        uint32_t dd = x > y ? x - y : y - x;
        if (c.topo == TOPO_TORUS && k - dd < dd) dd = k - dd;
        h += dd;
        a /= k;
        b /= k;
      }
      return h + 1;
    }
    case TOPO_FATTREE: {  // k-ary n-tree: up to the lowest common ancestor and down
      uint32_t lvl = 1;
      a /= k;
      b /= k;
      while (a != b && lvl < n) {
        a /= k;
        b /= k;
        ++lvl;
      }
      return 2 * lvl - 1;
    }
    default: {  // flattened butterfly (c terminals per router): one hop per differing dimension
      uint32_t h = 0;
      a /= (c.topo_conc ? c.topo_conc : 1);
      b /= (c.topo_conc ? c.topo_conc : 1);
      for (uint32_t d = 0; d < n; ++d) {
        h += (a % k) != (b % k);
        a /= k;
        b /= k;
      }
      return h + 1;
    }
  }
}

// refresh the period dividers after any change of per_* (config derivation,
// DVFS, checkpoint restore)
inline void cfg_set_divs(SimCfg& c) {
  c.dv_core = make_div64(c.per_core);
  c.dv_icnt = make_div64(c.per_icnt);
  c.dv_l2 = make_div64(c.per_l2);
  c.dv_dram = make_div64(c.per_dram);
  c.dv_epoch = make_div64(c.icnt_latency ? c.icnt_latency : 1);
}

// absolute femtoseconds of the start of core cycle `cyc`, and the core cycle
// holding femtosecond `fs` (floor) or starting at or after it (ceil)
SIM_HDI uint64_t core_fs(const SimCfg& c, uint64_t cyc) {
  return (uint64_t)((int64_t)c.clk_base_fs + ((int64_t)cyc - (int64_t)c.clk_base_cyc) * (int64_t)c.per_core);
}
SIM_HDI uint64_t core_cyc(const SimCfg& c, uint64_t fs) {
  if (fs >= c.clk_base_fs) return c.clk_base_cyc + fdiv(fs - c.clk_base_fs, c.dv_core);
  return c.clk_base_cyc - fdiv(c.clk_base_fs - fs + c.per_core - 1, c.dv_core);
}
SIM_HDI uint64_t core_cyc_ceil(const SimCfg& c, uint64_t fs) {
  if (fs >= c.clk_base_fs) return c.clk_base_cyc + fdiv(fs - c.clk_base_fs + c.per_core - 1, c.dv_core);
  return c.clk_base_cyc - fdiv(c.clk_base_fs - fs, c.dv_core);
}

// femtoseconds from injection complete to arrival: SM `sm` -> sub-partition `sub`
// (either direction; the topologies are symmetric)
SIM_HDI uint64_t icnt_pkt_lat_fs(const SimCfg& c, uint32_t sm, uint32_t sub) {
  if (c.icnt_mode != 1) return (uint64_t)c.icnt_latency * c.per_core;
  const uint32_t a = sm / (c.cores_per_cluster ? c.cores_per_cluster : 1);  // one node per cluster
  const uint32_t b = c.n_clusters + sub;                                  // then the sub-partitions
  const uint32_t r = icnt_routers(c, a, b);
  const uint64_t cyc = (uint64_t)r * c.hop_icnt + (uint64_t)(r + 1) * c.chan_icnt;
  const uint64_t fs = cyc * c.per_icnt;
  const uint64_t lo = (uint64_t)c.icnt_latency * c.per_core;  // never below the lookahead
  return fs > lo ? fs : lo;
}

SIM_HDI bool trace_sm_on(const SimCfg& c, uint32_t stream, uint32_t sm) {
  return (c.trace_mask & stream) && (c.trace_sm < 0 || (uint32_t)c.trace_sm == sm);
}
SIM_HDI bool trace_mem_on(const SimCfg& c, uint32_t stream, uint32_t ch) {
  return (c.trace_mask & stream) && (c.trace_mem < 0 || (uint32_t)c.trace_mem == ch);
}

// ---- helpers shared by both engines ----
SIM_HDI uint32_t unit_of(const SimCfg& c, uint8_t cls) {
  if (c.single_valu && (cls == OC_SFU || cls == OC_DP || cls == OC_INTP)) return U_SP;
  switch (cls) {
    case OC_LOAD: case OC_STORE: case OC_MEMBAR: return U_MEM;
    case OC_SFU: return U_SFU;
    case OC_DP: return c.unit_count[U_DP] ? U_DP : U_SFU;
    case OC_INTP: return c.unit_count[U_INT] ? U_INT : U_SP;
    case OC_TENSOR: return c.unit_count[U_TENSOR] ? U_TENSOR : U_SP;
    default:
      if (cls >= OC_SPEC1 && cls <= OC_SPEC8) {
        uint32_t u = U_SPEC1 + (cls - OC_SPEC1);
        return c.unit_count[u] ? u : (uint32_t)U_SP;
      }
      return U_SP;  // ALU, SP, BRANCH, BARRIER, EXIT, NOP
  }
}

}  // namespace asim
