// Device-resident data contracts shared by the CPU and GPU engines.
//
// The reference keeps each dynamic instruction as a heap-allocated
// `inst_trace_t` with a std::string opcode and a heap address block
// (trace_parser.h:55-79) and re-decodes it into a `trace_warp_inst_t` at issue
// (trace_driven.cc:151-381).  Here the whole kernel trace is decoded ONCE on
// the host into fixed 32-byte records that live in HBM for the duration of
// the simulated kernel (288 GB/GPU holds ~9e9 of them), so the cycle engine
// never parses text or allocates.
#pragma once
#include "hd.h"

namespace asim {

// ---- micro-architectural operation classes (reference: uarch_op_t,
// abstract_hardware_model.h:108-138, plus the trace-mode category map of
// ISA_Def/*_opcode.h) ----
enum OpCls : uint8_t {
  OC_ALU = 0,   // generic ALU (MOV, S2R, LDC, SHFL, ...)
  OC_SP,        // single precision FP
  OC_DP,        // double precision FP
  OC_SFU,       // transcendental / MUFU
  OC_TENSOR,    // matrix core (HMMA / MFMA)
  OC_INTP,      // integer pipe
  OC_LOAD,      // memory read (also atomics)
  OC_STORE,     // memory write
  OC_BRANCH,    // control flow
  OC_BARRIER,   // CTA barrier
  OC_MEMBAR,    // memory fence
  OC_EXIT,      // warp exit
  OC_NOP,
  OC_SPEC1,     // specialized units 1..8 (reference SPEC_UNIT_START_ID)
  OC_SPEC2,
  OC_SPEC3,
  OC_SPEC4,
  OC_SPEC5,
  OC_SPEC6,
  OC_SPEC7,
  OC_SPEC8,
  OC_COUNT
};

// execution unit types (one pipeline register set each)
enum Unit : uint8_t {
  U_SP = 0,
  U_DP,
  U_INT,
  U_SFU,
  U_TENSOR,
  U_MEM,
  U_SPEC1,  // .. U_SPEC8
  U_COUNT = U_SPEC1 + 8
};

enum Space : uint8_t {
  S_NONE = 0,
  S_GLOBAL,
  S_LOCAL,
  S_SHARED,
  S_CONST,
  S_TEX,
  S_PARAM,
};

enum InstFlags : uint8_t {
  F_BYPASS_L1 = 1,  // LDG.E.STRONG.GPU etc: served at L2 (trace_driven.cc:266-270)
  F_ATOMIC = 2,     // ATOM/RED/ATOMG: performed at L2
  F_MEM = 4,        // has an address record
  F_WAITCNT = 8,    // CDNA s_waitcnt: wait for all outstanding memory of the wave
};

// 32-byte decoded dynamic warp instruction.
struct TInst {
  uint32_t pc;
  uint32_t mem;     // index into TMem table or kNoMem
  uint64_t mask;    // active-thread mask (32 or 64 lanes)
  uint16_t opcode;  // global ISA opcode id (isa_tables) for stats/power
  uint8_t cls;      // OpCls
  uint8_t space;    // Space
  uint8_t dst[2];   // register+1, 0 = none  (reference adds 1: trace_driven.cc:225-240)
  uint8_t src[5];   // register+1, 0 = none  (5 sources: fixes reference defect D3)
  uint8_t width;    // bytes per thread for memory ops
  uint16_t lat;     // pipeline latency (cycles)
  uint8_t ii;       // initiation interval
  uint8_t flags;    // InstFlags
};
static_assert(sizeof(TInst) == 32, "TInst must stay 32 bytes");
constexpr uint32_t kNoMem = 0xffffffffu;

// Per-instruction address record.  Addresses of active lanes are either
// base + k*stride (k = rank among active lanes) or an explicit list (one
// u64 per ACTIVE lane, in lane order) starting at addrs[list].
struct TMem {
  uint64_t base;
  int32_t stride;
  uint32_t list;  // kNoMem -> base/stride form
};
static_assert(sizeof(TMem) == 16, "TMem must stay 16 bytes");

// warp instruction stream of one warp of one CTA: [begin, begin+count)
struct WStream {
  uint32_t begin;
  uint32_t count;
};

// ---- per-access record produced by the trace-ingest coalescer ----
// line (128B aligned) | sector mask (bits 0..3) | (bytes/4-1) in bits 4..6 is
// NOT packed: keep it simple and 16-byte aligned.
struct TAcc {
  uint64_t line;     // 128B-aligned line address
  uint16_t bytes;    // bytes touched (write packet size)
  uint8_t sectors;   // 32B sector mask
  uint8_t bank;      // L1 bank (precomputed)
  uint32_t pad;
};
static_assert(sizeof(TAcc) == 16, "TAcc must stay 16 bytes");

// Interconnect packet (32 B).  Time stamps are femtoseconds so that the
// four clock domains (core/icnt/L2/DRAM, reference gpu-sim.cc:1047-1062) are
// exact integers.
enum PktType : uint8_t {
  P_RD = 1,     // read request (sector mask)
  P_WR,         // write request
  P_ATOM,       // atomic request (returns data)
  P_RD_REPLY,
  P_WR_ACK,
  P_ATOM_REPLY,
};
struct Pkt {
  uint64_t addr;  // 128B-line aligned byte address
  uint64_t t;     // time the packet becomes visible at its destination (fs)
  uint32_t tag;   // requester cookie (SM side: load slot / mshr)
  uint16_t src;
  uint16_t dst;
  uint16_t size;  // bytes on the wire
  uint8_t type;
  uint8_t sectors;  // 32B-sector mask within the line
  uint32_t aux;
};
static_assert(sizeof(Pkt) == 32, "Pkt must stay 32 bytes");

// Device view of one simulated kernel.
struct KernelDesc {
  uint32_t uid;
  uint32_t n_cta;
  uint32_t warps_per_cta;
  uint32_t threads_per_cta;
  uint32_t shmem_per_cta;
  uint32_t regs_per_thread;
  uint32_t cta_per_sm;  // resource-limited CTA slots per SM for this kernel
  uint32_t grid[3];
  uint32_t block[3];
  uint32_t stream;
  uint32_t l1_sets, l1_assoc;  // adaptive L1 geometry chosen for this kernel
  uint32_t stop_when_issued;   // cut to the -gpgpu_max_cta remainder: the run ends once all CTAs issued
  uint32_t flush_l1;           // bit 0 -gpgpu_flush_l1_cache: SMs drop their L1 when the kernel starts;
                               // bit 1 -sim_sqc_invalidate_at_launch: and their instruction / scalar caches
  // per-CTA SM resources (shader_core_ctx::occupy_shader_resource_1block):
  // warp-padded threads, registers, and the shared-memory capacity of the
  // carve-out chosen for this kernel
  uint32_t thr_cta, regs_cta, shmem_cap, pad_k;
  // trace residency (GPU engine, -gpu_trace_window): instruction, access and
  // CTA-stream indices are taken modulo ring capacities (masks: all ones when
  // the whole kernel is resident) and CTAs >= cta_avail are not uploaded yet
  // (epoch_decide ends the launch before a dispatch could need one)
  uint32_t imask, amask, cmask, cta_avail;
  uint64_t ready_cycle;        // launch + kernel/CTA launch latency: first CTA dispatch
  uint64_t shmem_base;
  uint64_t local_base;
  uint64_t n_insts;
  const TInst* insts;
  const TAcc* accs;        // coalesced access table (inst.mem indexes it)
  const WStream* streams;  // [n_cta * warps_per_cta]
  uint64_t pad_p;
};

// Concurrent kernels (reference gpgpu_sim::m_running_kernels, gpu-sim.cc:805-900,
// and the stream window of gpu-simulator/main.cc:74-115).  A warp's
// instruction indices (w_next / w_head / w_end) carry the kernel slot in
// their top bits, so the fetch / issue paths index one merged instruction
// space with no per-warp kernel lookup beyond the slot's base pointer.
constexpr int kMaxConc = 8;
constexpr uint32_t kSlotShift = 29;
constexpr uint32_t kIdxMask = (1u << kSlotShift) - 1;
struct KernelTab {
  KernelDesc k[kMaxConc];
  uint32_t active;  // bit k: slot k holds a launched kernel that has not completed
  uint32_t mix;     // -gpgpu_concurrent_kernel_sm: one SM may hold CTAs of several kernels
  uint64_t pad[3];
};
SIM_HDI const TInst& inst_at(const KernelTab& kt, uint32_t gi) {
  const KernelDesc& k = kt.k[gi >> kSlotShift];
  return k.insts[gi & kIdxMask & k.imask];
}

}  // namespace asim
