// Trace ingest: command lists, kernel headers, instruction streams.
//
// Compatible readers for the reference's text formats (kernelslist.g,
// kernel-N.traceg: trace_parser.cc:220-447) plus this project's binary
// columnar format (".asimk", written by the tracer/generator, memory-mappable,
// config independent).  All formats decode into the same host arrays, which
// are then coalesced for a given SimCfg and uploaded once per kernel.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../model/sm.h"

namespace asim {

enum CmdType : uint8_t {
  CMD_KERNEL = 1,
  CMD_MEMCPY_HTOD,
  CMD_MEMCPY_DTOH,
  CMD_COLL_INIT,      // ncclCommInitAll / rcclCommInitRank
  CMD_COLL_DESTROY,   // ncclCommDestroy
  CMD_GROUP_START,    // ncclGroupStart
  CMD_GROUP_END,      // ncclGroupEnd
  CMD_COLLECTIVE,     // ncclAllReduce / AllGather / ReduceScatter / Broadcast / AllToAll ...
  CMD_EVENT_RECORD,   // hipEventRecord,event=E,stream=S: fires when S's earlier work is done
  CMD_EVENT_WAIT,     // hipStreamWaitEvent,stream=S,event=E: S waits for the latest earlier record of E
};

struct Command {
  CmdType type;
  std::string text;   // original line (or resolved kernel path)
  uint64_t addr = 0;  // memcpy
  uint64_t bytes = 0; // memcpy / collective payload bytes per rank
  // collective description (fixes the reference's dropped arguments, D6/§2.11)
  std::string coll;   // AllReduce, AllGather, ReduceScatter, Broadcast, Reduce, AllToAll, SendRecv
  uint64_t count = 0;
  uint32_t dtype_bytes = 4;
  std::string redop;
  int32_t root = -1;
  int32_t nranks = 1;
  uint64_t stream = 0;
  uint64_t event = 0;  // event record / wait
};

// Parse a kernelslist(.g) file.  Kernel paths are resolved relative to it.
std::vector<Command> parse_commandlist(const std::string& path);
// Parse one collective line "ncclAllReduce[,count=..,dtype=..,op=..,nranks=..]"
Command parse_collective_line(const std::string& line);

struct KernelHeader {
  std::string name = "Empty";
  uint32_t id = 0;
  uint32_t grid[3] = {1, 1, 1};
  uint32_t block[3] = {1, 1, 1};
  uint32_t shmem = 0;
  uint32_t nregs = 0;
  uint64_t stream = 0;
  uint32_t binary_version = 0;
  uint32_t trace_version = 0;
  std::string tracer_version;
  uint64_t shmem_base = 0;
  uint64_t local_base = 0;
  uint32_t warp_size = 32;
};

// Decoded (not yet coalesced) kernel trace.
struct HostKernel {
  KernelHeader h;
  uint32_t warps_per_cta = 0;
  uint32_t n_cta = 0;
  std::vector<TInst> insts;   // inst.mem -> index into mems, inst.width = bytes/thread
  std::vector<TMem> mems;
  std::vector<uint64_t> addrs;
  std::vector<WStream> streams;  // [n_cta * warps_per_cta]
  uint64_t thread_insts = 0;
  uint64_t warp_insts = 0;
  uint32_t unknown_opcodes = 0;
};

class KernelReader;  // per-CTA reader of a text kernel trace (below)

// index widths of a host-streamed kernel: warp stream begins are kept modulo
// 2^28 (begin + count stays below the engines' 2^29 slot field), access
// indices modulo 2^31 (never kNoMem); the rings are at most that large
constexpr uint64_t kStreamInstMask = (1ull << 28) - 1;
constexpr uint64_t kStreamAccMask = (1ull << 31) - 1;

// Coalesced kernel ready for a cycle engine (inst.mem -> first TAcc,
// inst.width -> number of accesses, or shared-memory conflict degree).
//
// Host streaming (-trace_host_budget_mb): a ReadyKernel with a reader `src`
// holds only the CTAs [cta_lo, cta_hi) of the kernel -- parsed and ingested
// from the trace file as the engines' trace windows advance
// (engine/trace_window.h), dropped once every SM is done with them -- so the
// host's trace memory is bounded by the window, not by the kernel (the
// reference reads thread blocks from the file as CTAs issue,
// gpu-simulator/trace-parser/trace_parser.cc:387-447).  Indices stay global:
// insts[0] is instruction `ibase`, accs[0] access `abase`, streams[0] the
// first warp of CTA cta_lo; ib / ab give the first instruction / access of
// CTAs cta_lo..cta_hi.  Without a reader the whole kernel is held (all of
// these are 0 / empty).
struct ReadyKernel {
  KernelHeader h;
  uint32_t warps_per_cta = 0;
  uint32_t n_cta = 0;
  std::vector<TInst> insts;
  std::vector<TAcc> accs;
  std::vector<WStream> streams;
  uint64_t thread_insts = 0;
  uint64_t warp_insts = 0;
  std::shared_ptr<KernelReader> src;
  uint32_t cta_lo = 0, cta_hi = 0;
  uint64_t ibase = 0, abase = 0;
  std::vector<uint64_t> ib, ab;
  uint64_t host_peak_bytes = 0;  // largest host footprint of the resident CTAs (streamed kernels)
  bool streamed() const { return (bool)src; }
  // make CTAs [lo, hi) resident: parse forward as needed, drop CTAs below lo
  void resident(uint32_t lo, uint32_t hi);
  uint64_t host_bytes() const {
    return insts.capacity() * sizeof(TInst) + accs.capacity() * sizeof(TAcc) + streams.capacity() * sizeof(WStream) +
           (ib.capacity() + ab.capacity()) * sizeof(uint64_t);
  }
};

// Sequential reader of a text kernel trace (.traceg), one thread block at a
// time, each ingested (coalesced) as soon as it is read.  Thread blocks must
// come in linear-id order (the format's rule), else it throws.
class KernelReader {
 public:
  KernelReader(const std::string& path, const SimCfg& c);
  ~KernelReader();
  const KernelHeader& header() const;
  uint32_t n_cta() const;
  uint32_t warps_per_cta() const;
  // the next CTA's instructions / accesses / warp streams appended to the
  // vectors; global indices continue from `ibase + insts.size()` (instruction)
  // and `abase + accs.size()` (access)
  void next_cta(std::vector<TInst>& insts, std::vector<TAcc>& accs, std::vector<WStream>& streams, uint64_t ibase,
                uint64_t abase);
  uint32_t ctas_read() const;

 private:
  struct Impl;
  Impl* p_;
};

// A streamed ReadyKernel for the trace at `path` (text format), nothing
// resident yet
ReadyKernel open_streamed_kernel(const std::string& path, const SimCfg& c);

// Synthetic streaming-copy kernel: the memory traffic of a collective on one
// GPU (RCCL runs collectives as kernels that read the local send buffer and
// write the receive buffer while the link moves the data).  n_cta workgroups
// of `warps` waves; every wave loads its share of [src, src + rd_bytes) and
// stores its share of [dst, dst + wr_bytes) in wave-wide 16 B-per-lane
// accesses, four loads in flight before the stores that forward them.
HostKernel make_copy_kernel(const std::string& name, uint32_t binary_version, uint32_t warp_size, uint32_t n_cta,
                            uint32_t warps, uint64_t src, uint64_t rd_bytes, uint64_t dst, uint64_t wr_bytes,
                            uint64_t stream);

// header only (cheap); used by the command loop before the body is needed
KernelHeader read_kernel_header(const std::string& path);
HostKernel load_kernel(const std::string& path);  // text (.traceg/.trace) or binary (.asimk)
HostKernel load_kernel_text(const std::string& path);
HostKernel load_kernel_binary(const std::string& path);
void save_kernel_binary(const HostKernel& k, const std::string& path);
void save_kernel_text(const HostKernel& k, const std::string& path);

// ISA decode of one mnemonic (e.g. "LDG.E.64.STRONG.GPU") for an
// architecture selected by the kernel's binary version (SASS: 30..90,
// CDNA: 900+, e.g. 950 = gfx950).
struct OpInfo {
  uint16_t opcode;
  uint8_t cls;
  uint8_t space;
  uint8_t flags;
  uint8_t width;      // bytes per thread (memory)
  uint8_t half_ii;    // FP16x2: half initiation interval
  bool known;
};
OpInfo decode_opcode(const std::string& op, uint32_t binary_version);
const std::string& opcode_name(uint16_t id);
uint32_t opcode_count();

// Coalescing (host reference of the trace-ingest coalescer; same function is
// run lane-parallel by the HIP ingest kernel).
ReadyKernel coalesce_kernel(const HostKernel& k, const SimCfg& c);
// ingest steps of one instruction (coalesce_kernel is built from them; the
// MI355X coalescer, engine/ingest_mfma.hip, runs the address-dependent ones
// on the device and these on the host)
enum IngestKind : uint8_t { IK_DONE = 0, IK_SCALAR, IK_SMEM, IK_GMEM };
IngestKind ingest_prepare(TInst& in, const SimCfg& c);  // latency / ii, address-less fixes
void ingest_scalar(TInst& in, const SimCfg& c, uint64_t name_hash, std::vector<TAcc>& accs);
// sorted 128B-line accesses of one global instruction (<= kMaxAccess into out)
uint32_t coalesce_lanes(const uint64_t* lane, uint64_t mask, uint32_t width, uint32_t ws, const SimCfg& c, TAcc* out);
void ingest_finish_global(TInst& in, const TAcc* a, uint32_t n, std::vector<TAcc>& accs);
void ingest_lane_addresses(const HostKernel& k, const TInst& in, uint64_t* out, uint32_t ws);
ReadyKernel ingest_shell(const HostKernel& k);  // everything but the coalesced instructions
struct IngestStats {
  uint64_t smem_jobs = 0, smem_host = 0;  // shared-memory instructions: on the device / fell back to the host
  uint64_t gmem_jobs = 0, gmem_host = 0;  // global instructions: on the device / fell back to the host
  uint64_t mfma = 0;                      // matrix-core instructions issued
  double device_s = 0, total_s = 0;
};
// MI355X coalescer (bank-by-row and line-by-sector occupancy matrices on the
// matrix cores); false when no HIP device / build
bool gpu_coalesce_kernel(const HostKernel& k, const SimCfg& c, int device, ReadyKernel& out, IngestStats* st);
// device >= 0: coalesce on that HIP device (bit-identical to coalesce_kernel),
// else, or when it is unavailable, on the host
ReadyKernel ingest_kernel(const HostKernel& k, const SimCfg& c, int device = -1, IngestStats* st = nullptr);
int gpu_current_device();  // the calling thread's HIP device (-1: none / CPU-only build)

// shared-memory bank-conflict degree of one warp access
// CDNA4 LDS banking of one ds_* instruction: its lane groups (one LDS cycle
// each) and bank count
struct LdsGroups {
  uint32_t n;          // lane groups (<= 8)
  uint32_t nb;         // banks: 32 or 64
  uint64_t lanes[8];   // lanes of each group
};
const LdsGroups* lds_groups_for(const std::string& lower_case_opcode);
// the groups of `opcode` with -gpgpu_shmem_cdna_lane_groups on a wave64 trace, else nullptr
const LdsGroups* lds_groups(const SimCfg& c, uint16_t opcode, uint32_t warp_size);
// groups == nullptr: the GPGPU-Sim model (-gpgpu_shmem_warp_parts, banks,
// limited broadcast); else 1 + the CDNA4 extra cycles over the groups
uint32_t smem_conflict_degree(const uint64_t* addr, uint64_t mask, uint32_t width, const SimCfg& c, uint32_t warp_size,
                              const LdsGroups* groups = nullptr);

}  // namespace asim
