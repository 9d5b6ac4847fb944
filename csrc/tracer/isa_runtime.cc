// Host runtime of the automatic gfx950 ISA tracer (linked into executables
// built by accel_sim_framework_distributed_amd/isatrace/build.py).
//
// Reference: the host half of the NVBit tracer -- nvbit_at_cuda_event
// (util/tracer_nvbit/tracer_tool/tracer_tool.cu:380-506) resets the device
// channel per launch, waits for the kernel, and the receiver thread
// (:508-700) turns the pushed records into the kernel-N.traceg text format
// (PC, active mask, registers, opcode, addresses), plus kernelslist.g with
// MemcpyHtoD lines (:369-378).
//
// Here the instrumented code object (isatrace/rewrite.py) appends per-wave
// record streams to 8 KB chunks.  By default the chunks form a ring in
// coherent host memory that a drain thread empties while the kernel runs
// (closed chunks are spilled to a file next to the trace and their slots
// handed back), so the trace of one kernel is bounded by disk, not by a
// buffer -- the reference's device channel + receiver thread
// (util/tracer_nvbit/nvbit_release/core/utils/channel.hpp:56-116,161-253).
// ASIM_TRACE_BUF_MB selects the older one-device-buffer mode instead (faster
// for small kernels; a kernel that outgrows it fails the run).  A capture is
// lossless or the traced program exits with status 5 (fail_run): no partial
// kernel trace is ever written.
// This runtime
//  * interposes __hipRegisterFatBinary / __hipRegisterFunction to register
//    the probes' control block (device global __asim_tctl) and learn kernel
//    names, and hipLaunchKernel to arm the buffer, launch, wait and decode;
//  * expands each wave's segment / memory records with the static map
//    (<exe>.asimisa: every segment's instructions with real byte offsets,
//    registers and memory widths) into trace lines;
//  * writes kernel-N.traceg (format v4, wavefront size 64, binary version
//    950), kernelslist.g (+ MemcpyHtoD lines from hipMemcpy) and stats.csv.
// Environment: ASIM_TRACE_DIR (enables tracing), ASIM_TRACE_KERNEL_START/END
// (1-based launch range), ASIM_TRACE_RING_MB / _KB (host ring, default 256 MB,
// rounded down to a power-of-two number of chunks), ASIM_TRACE_SPIN_LIMIT
// (slot polls before a waiting wave gives up: the run then fails, status 5,
// and no partial trace is written), ASIM_TRACE_DRAIN_DELAY_US (test hook), ASIM_TRACE_BUF_MB (device-buffer
// mode instead of the ring), ASIM_ISA_MAP (map path, default <exe>.asimisa),
// ASIM_TRACE_GPU_ID / GPU_TRACE_ID (trace only the launches on that HIP
// device, files kernel-<id>_<gpu>.traceg: the reference's per-device filter
// and naming, tracer_tool.cu:115-116,303-316,442-445).  "{rank}" in
// ASIM_TRACE_DIR becomes the process's rank (RANK, OMPI_COMM_WORLD_RANK,
// SLURM_PROCID or LOCAL_RANK), so every rank of a multi-process job writes
// its own trace directory.  ASIM_TRACE_SNAPSHOT=1: the silicon-checkpoint
// allocation tracking (hipMalloc / hipFree interposed; after every traced
// kernel kernel-<id>.allocs lists the live allocations and
// kernel-<id>_alloc-<n>.bin holds their contents, up to
// ASIM_TRACE_SNAPSHOT_MAX_MB per kernel).  ASIM_TRACE_BBV=1: per-wave
// basic-block vectors of every traced kernel (kernel-<id>.bbv).
#include <filesystem>
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

constexpr uint32_t kTagMem = 0x80000000u, kTagChunk = 0xC0000000u, kTagClose = 0xE0000000u;
// 16-byte units per chunk: from the map header (isatrace/rewrite.py CHUNK_UNITS)
uint32_t kChunkUnits = 512;

struct Ctl {  // must match the probes (isatrace/rewrite.py)
  uint64_t buf;         // @0  ring (device view of the host ring) or device buffer
  uint32_t next_chunk;  // @8  tickets handed out
  uint32_t n_chunks;    // @12 device-buffer mode: chunks in the buffer
  uint32_t mask;        // @16 ring mode: slots - 1 (0 = device-buffer mode)
  uint32_t shift;       // @20 ring mode: log2(slots)
  uint32_t spin_limit;  // @24 ring mode: slot polls before a wave gives up (0: the probes' default)
  uint32_t pad;
};
static_assert(sizeof(Ctl) == 32, "control block layout");

struct SInst {
  uint32_t pc;
  int32_t mem;
  std::string text;  // "<ndst> <dsts> <mnemonic> <nsrc> <srcs>" (trace line middle)
  int width;
};
struct KMap {
  std::vector<std::vector<SInst>> segs;  // seg id - 1
  uint32_t lds = 0, vgprs = 32;
};

#define RT_HIP(x)                                                                                    \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      fprintf(stderr, "asim isa tracer: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                                             \
      exit(3);                                                                                       \
    }                                                                                                \
  } while (0)

struct Tracer {
  bool enabled = false;
  std::string dir;
  long kstart = 1, kend = 1L << 40;
  int gpu_id = -1;  // -1: every device
  long next_id = 0;
  size_t buf_bytes = 0;           // device-buffer mode when set
  size_t ring_bytes = 256ull << 20;
  // slot polls (each ~1 us: a system-scope load + s_sleep) before a waiting
  // wave gives up; it exists only so a stalled host cannot hang the GPU
  uint32_t spin_limit = 1u << 22;
  uint32_t drain_delay_us = 0;  // test hook: slow the drain thread down
  struct Ring {
    uint8_t* host = nullptr;  // coherent host memory
    uint8_t* dev = nullptr;   // the same memory as the GPU addresses it
    uint32_t slots = 0, shift = 0;
  };
  std::unordered_map<int, Ring> rings;  // one ring per device
  struct DevBuf {
    uint8_t* ptr = nullptr;
    uint32_t last_used = 0;  // chunks written by the previous traced launch (re-zeroed)
  };
  std::unordered_map<int, DevBuf> bufs;  // one trace buffer per device (launch device's HBM)
  std::mutex mu;
  std::unordered_map<std::string, KMap> maps;
  std::unordered_map<const void*, std::string> names;
  std::vector<Ctl*> shadows;  // one device __asim_tctl per registered code object
  // silicon-checkpoint allocation tracking (reference
  // util/tracer_nvbit/others/silicon_checkpoint_tool/checkpoint/checkpoint.cu:198-290):
  // live device allocations (address -> allocation number, bytes); with
  // ASIM_TRACE_SNAPSHOT set, after every traced kernel each live allocation's
  // contents go to kernel-<id>_alloc-<n>.bin and the list to kernel-<id>.allocs
  struct Alloc {
    uint32_t num;
    size_t bytes;
  };
  std::map<uintptr_t, Alloc> allocs;
  uint32_t alloc_count = 0;
  bool snapshot = false;
  bool bbv = false;  // ASIM_TRACE_BBV: per-wave basic-block vectors (kernel-<id>.bbv)
  size_t snapshot_max = 1ull << 30;  // bytes per kernel snapshot (ASIM_TRACE_SNAPSHOT_MAX_MB)

  Tracer() {
    const char* d = getenv("ASIM_TRACE_DIR");
    if (!d || !*d) return;
    enabled = true;
    dir = d;
    for (size_t at; (at = dir.find("{rank}")) != std::string::npos;) {
      const char* r = nullptr;
      for (const char* v : {"RANK", "OMPI_COMM_WORLD_RANK", "SLURM_PROCID", "LOCAL_RANK"})
        if ((r = getenv(v)) && *r) break;
      dir.replace(at, 6, r && *r ? r : "0");
    }
    if (const char* s = getenv("ASIM_TRACE_GPU_ID")) gpu_id = atoi(s);
    else if (const char* s2 = getenv("GPU_TRACE_ID")) gpu_id = atoi(s2);
    std::error_code ec;
    std::filesystem::create_directories(dir, ec);
    FILE* kl = fopen((dir + "/kernelslist.g").c_str(), "w");
    if (!kl) {
      fprintf(stderr, "asim isa tracer: cannot write %s/kernelslist.g (%s); tracing disabled\n", dir.c_str(),
              ec ? ec.message().c_str() : "open failed");
      enabled = false;
      return;
    }
    fclose(kl);
    FILE* f = fopen((dir + "/stats.csv").c_str(), "w");
    if (f) {
      fprintf(f, "kernel id, kernel name, grid_dim, block_dim, #warp insts, #thread insts\n");
      fclose(f);
    }
    if (const char* s = getenv("ASIM_TRACE_KERNEL_START")) kstart = atol(s);
    if (const char* s = getenv("ASIM_TRACE_KERNEL_END")) kend = atol(s);
    if (const char* s = getenv("ASIM_TRACE_BUF_MB")) buf_bytes = (size_t)atol(s) << 20;
    if (const char* s = getenv("ASIM_TRACE_RING_MB")) ring_bytes = (size_t)atol(s) << 20;
    if (const char* s = getenv("ASIM_TRACE_RING_KB")) ring_bytes = (size_t)atol(s) << 10;
    if (const char* s = getenv("ASIM_TRACE_SPIN_LIMIT")) spin_limit = (uint32_t)std::max(1L, atol(s));
    if (const char* s = getenv("ASIM_TRACE_DRAIN_DELAY_US")) drain_delay_us = (uint32_t)atol(s);
    if (const char* s = getenv("ASIM_TRACE_SNAPSHOT")) snapshot = *s && *s != '0';
    if (const char* s = getenv("ASIM_TRACE_BBV")) bbv = *s && *s != '0';
    if (const char* s = getenv("ASIM_TRACE_SNAPSHOT_MAX_MB")) snapshot_max = (size_t)atol(s) << 20;
    std::string mp;
    if (const char* s = getenv("ASIM_ISA_MAP")) {
      mp = s;
    } else {
      char exe[4096];
      ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
      if (n > 0) {
        exe[n] = 0;
        mp = std::string(exe) + ".asimisa";
      }
    }
    load_map(mp);
  }

  void load_map(const std::string& path) {
    std::ifstream in(path);
    if (!in) {
      fprintf(stderr, "asim isa tracer: no instruction map %s (tracing disabled)\n", path.c_str());
      enabled = false;
      return;
    }
    std::string line;
    KMap* k = nullptr;
    std::vector<SInst>* seg = nullptr;
    while (std::getline(in, line)) {
      if (line.rfind("ASIMISA", 0) == 0) {
        std::istringstream hs(line);
        std::string tag;
        int ver = 0;
        uint32_t cu = 0;
        hs >> tag >> ver >> cu;
        if (cu) kChunkUnits = cu;
        continue;
      }
      if (line.empty()) continue;
      std::istringstream ss(line);
      if (line[0] == 'K' && line[1] == ' ') {
        std::string tag, name;
        size_t nseg = 0, nmem = 0;
        ss >> tag >> name >> nseg >> nmem;
        k = &maps[name];
        k->segs.assign(nseg, {});
        ss >> k->lds >> k->vgprs;
        seg = nullptr;
      } else if (line[0] == 'S' && line[1] == ' ') {
        std::string tag;
        size_t id = 0, n = 0;
        ss >> tag >> id >> n;
        if (k && id >= 1 && id <= k->segs.size()) seg = &k->segs[id - 1];
      } else if (seg) {
        SInst si;
        std::string pc;
        ss >> pc >> si.mem;
        si.pc = (uint32_t)strtoul(pc.c_str(), nullptr, 16);
        // rest of the line: ndst dsts mnemonic nsrc srcs width
        std::string rest;
        std::getline(ss, rest);
        size_t b = rest.find_first_not_of(' ');
        rest = b == std::string::npos ? "" : rest.substr(b);
        size_t e = rest.find_last_of(' ');
        si.width = atoi(rest.c_str() + e + 1);
        si.text = rest.substr(0, e);
        seg->push_back(si);
      }
    }
  }

  bool traced(long id) const { return enabled && id >= kstart && id <= kend; }
  // the launch / copy happens on a device this process traces
  bool on_traced_device() const {
    if (gpu_id < 0) return true;
    int dev = 0;
    return hipGetDevice(&dev) == hipSuccess && dev == gpu_id;
  }
  std::string kernel_file(long id) const {
    return "kernel-" + std::to_string(id) + (gpu_id >= 0 ? "_" + std::to_string(gpu_id) : std::string()) + ".traceg";
  }

  void append(const std::string& file, const std::string& s) {
    FILE* f = fopen((dir + "/" + file).c_str(), "a");
    if (f) {
      fprintf(f, "%s\n", s.c_str());
      fclose(f);
    }
  }
};

Tracer& T() {
  static Tracer t;
  return t;
}

struct Wave {
  std::vector<std::pair<uint32_t, uint32_t>> chunks;  // (seq, chunk index)
};

void write_kernel(Tracer& t, long id, const std::string& name, const KMap& km, dim3 g, dim3 b, size_t shmem,
                  const uint8_t* host, uint32_t used) {
  // group chunks by wave: (wg z, wg y, wg x, packed tid of the first lane)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, Wave> waves;
  const size_t cb = (size_t)kChunkUnits * 16;
  for (uint32_t c = 0; c < used; ++c) {
    const uint32_t* u = reinterpret_cast<const uint32_t*>(host + c * cb);
    if ((u[0] & kTagChunk) != kTagChunk) continue;
    waves[std::make_tuple(u[3], u[2], u[1], u[4])].chunks.push_back({u[0] & ~kTagChunk, c});
  }
  const std::string fn = t.kernel_file(id);
  FILE* f = fopen((t.dir + "/" + fn).c_str(), "w");
  if (!f) {
    fprintf(stderr, "asim isa tracer: cannot write %s\n", fn.c_str());
    exit(3);
  }
  fprintf(f, "-kernel name = %s\n-kernel id = %ld\n-grid dim = (%u,%u,%u)\n-block dim = (%u,%u,%u)\n", name.c_str(),
          id, g.x, g.y, g.z, b.x, b.y, b.z);
  fprintf(f, "-shmem = %zu\n-nregs = %u\n-binary version = 950\n-wavefront size = 64\n-hip stream id = 0\n",
          shmem + km.lds, km.vgprs);
  fprintf(f, "-shmem base_addr = 0x0\n-local mem base_addr = 0x0\n-rocprofiler version = asim_isa_tracer\n");
  fprintf(f, "-accelsim tracer version = 4\n\n");
  fprintf(f, "#traces format = PC mask dest_num reg_dests opcode src_num reg_srcs mem_width mem_addresses\n\n");
  uint64_t winsts = 0, tinsts = 0;
  long bad = 0;
  std::vector<std::string> lines;
  // basic-block vectors from the instrumented binary (reference bbv_tool,
  // util/tracer_nvbit/others/bbv_tool/bbv_count/bbv_count.cu:88-143,320-340):
  // the rewriter's segments are the basic blocks (cut at every branch, label
  // and EXEC write); each execution adds its active-thread count
  std::vector<std::vector<uint64_t>> bbv_rows;
  auto it = waves.begin();
  while (it != waves.end()) {
    const uint32_t cz = std::get<0>(it->first), cy = std::get<1>(it->first), cx = std::get<2>(it->first);
    fprintf(f, "#BEGIN_TB\n\nthread block = %u,%u,%u\n\n", cx, cy, cz);
    // waves of this CTA in wave-index order
    std::vector<std::pair<uint32_t, Wave*>> ws;
    for (; it != waves.end() && std::get<0>(it->first) == cz && std::get<1>(it->first) == cy &&
           std::get<2>(it->first) == cx;
         ++it) {
      const uint32_t p = std::get<3>(it->first);
      const uint32_t tx = p & 0x3ff, ty = (p >> 10) & 0x3ff, tz = (p >> 20) & 0x3ff;
      const uint32_t flat = tx + ty * b.x + tz * b.x * b.y;
      ws.push_back({flat / 64, &it->second});
    }
    std::sort(ws.begin(), ws.end(), [](auto& x, auto& y) { return x.first < y.first; });
    for (auto& w : ws) {
      std::sort(w.second->chunks.begin(), w.second->chunks.end());
      lines.clear();
      // flatten the wave's records
      std::vector<const uint32_t*> recs;
      for (auto& ch : w.second->chunks) {
        const uint32_t* base = reinterpret_cast<const uint32_t*>(host + ch.second * cb);
        uint32_t u = 2;
        while (u < kChunkUnits) {
          const uint32_t* r = base + u * 4;
          if (r[0] == 0) break;
          recs.push_back(r);
          u += (r[0] & kTagMem) ? 33 : 1;
        }
      }
      size_t ri = 0;
      char buf[160];
      std::vector<uint64_t> bbv_row(t.bbv ? km.segs.size() : 0, 0);
      while (ri < recs.size()) {
        const uint32_t* r = recs[ri++];
        if (r[0] & kTagMem) {  // a memory record outside its segment: stream out of sync
          ++bad;
          continue;
        }
        const uint32_t sid = r[0];
        if (sid == 0 || sid > km.segs.size()) {
          ++bad;
          continue;
        }
        const uint64_t exec = (uint64_t)r[2] | (uint64_t)r[3] << 32;
        if (t.bbv) bbv_row[sid - 1] += (uint64_t)__builtin_popcountll(exec);
        for (const SInst& si : km.segs[sid - 1]) {
          uint64_t m = exec;
          const uint64_t* addrs = nullptr;
          if (si.mem >= 0) {
            if (ri < recs.size() && recs[ri][0] == (kTagMem | (uint32_t)si.mem)) {
              const uint32_t* mr = recs[ri++];
              m = (uint64_t)mr[2] | (uint64_t)mr[3] << 32;
              addrs = reinterpret_cast<const uint64_t*>(mr + 4);
            } else {
              ++bad;
            }
          }
          std::string ln;
          snprintf(buf, sizeof(buf), "%04x %016llx ", si.pc, (unsigned long long)m);
          ln = buf;
          ln += si.text;
          if (si.mem >= 0 && si.width) {
            snprintf(buf, sizeof(buf), " %d 0", si.width);
            ln += buf;
            if (addrs)
              for (int l = 0; l < 64; ++l)
                if ((m >> l) & 1ull) {
                  snprintf(buf, sizeof(buf), " 0x%llx", (unsigned long long)addrs[l]);
                  ln += buf;
                }
          } else {
            ln += " 0";
          }
          lines.push_back(ln);
          tinsts += (uint64_t)__builtin_popcountll(m);
        }
      }
      winsts += lines.size();
      if (t.bbv) bbv_rows.push_back(std::move(bbv_row));
      fprintf(f, "warp = %u\ninsts = %zu\n", w.first, lines.size());
      for (auto& l : lines) fprintf(f, "%s\n", l.c_str());
    }
    fprintf(f, "\n#END_TB\n\n");
  }
  fclose(f);
  if (t.bbv) {
    // reference layout: kernel name, waves, basic blocks, one row per wave
    const std::string bn = fn.substr(0, fn.rfind('.')) + ".bbv";
    FILE* bf = fopen((t.dir + "/" + bn).c_str(), "w");
    if (bf) {
      fprintf(bf, "%s\n%zu\n%zu\n", name.c_str(), bbv_rows.size(), km.segs.size());
      for (const auto& row : bbv_rows) {
        for (uint64_t v : row) fprintf(bf, "%llu ", (unsigned long long)v);
        fprintf(bf, "\n");
      }
      fclose(bf);
    }
  }
  if (bad) fprintf(stderr, "asim isa tracer: kernel %ld (%s): %ld records out of sequence\n", id, name.c_str(), bad);
  t.append("kernelslist.g", fn);
  char s[512];
  snprintf(s, sizeof(s), "kernel-%ld, %s, (%u,%u,%u), (%u,%u,%u), %llu, %llu", id, name.c_str(), g.x, g.y, g.z, b.x,
           b.y, b.z, (unsigned long long)winsts, (unsigned long long)tinsts);
  t.append("stats.csv", s);
}

// ---- streaming ring (isatrace/rewrite.py module docstring: the protocol)
struct Spill {
  FILE* f = nullptr;
  uint32_t chunks = 0;
  std::vector<uint8_t> tmp;
};

// copy one chunk out (the close marker cleared: record parsing stops at a
// zero unit)
void spill_chunk(const uint8_t* slot, size_t cb, Spill& sp) {
  sp.tmp.assign(slot, slot + cb);
  memset(sp.tmp.data() + cb - 16, 0, 16);
  if (fwrite(sp.tmp.data(), 1, cb, sp.f) != cb) {
    fprintf(stderr, "asim isa tracer: spill write failed\n");
    exit(3);
  }
  ++sp.chunks;
}

// one pass of the drain thread over the ring: every chunk its wave has
// closed is copied out, zeroed and handed to the slot's next generation
size_t drain_closed(const Tracer::Ring& r, Spill& sp) {
  const size_t cb = (size_t)kChunkUnits * 16;
  size_t n = 0;
  for (uint32_t s = 0; s < r.slots; ++s) {
    uint8_t* p = r.host + (size_t)s * cb;
    if (*reinterpret_cast<volatile const uint32_t*>(p + cb - 16) != kTagClose) continue;
    std::atomic_thread_fence(std::memory_order_acquire);
    volatile uint32_t* gen = reinterpret_cast<volatile uint32_t*>(p + 28);  // unit 1, word 3
    const uint32_t g = *gen;
    spill_chunk(p, cb, sp);
    memset(p, 0, 28);
    memset(p + 32, 0, cb - 32);
    std::atomic_thread_fence(std::memory_order_release);
    *gen = g + 1;
    ++n;
  }
  return n;
}

// after the kernel: every chunk still holding records (closed or not), then
// all touched slots back to generation 0 for the next launch
void drain_final(const Tracer::Ring& r, uint32_t tickets, Spill& sp) {
  const size_t cb = (size_t)kChunkUnits * 16;
  const uint32_t touched = tickets >= r.slots ? r.slots : tickets;
  for (uint32_t s = 0; s < touched; ++s) {
    uint8_t* p = r.host + (size_t)s * cb;
    if ((reinterpret_cast<const uint32_t*>(p)[0] & kTagChunk) == kTagChunk) spill_chunk(p, cb, sp);
    memset(p, 0, cb);
  }
}

// After a traced kernel (already synchronised): the live allocations' list
// and, with ASIM_TRACE_SNAPSHOT, their contents (the reference's per-kernel
// memory snapshot, checkpoint.cu:258-282; binary instead of one decimal
// text token per byte).  Called with the tracer lock held.
void snapshot_allocs(Tracer& t, long id, const std::string& suffix) {
  if (!t.snapshot) return;
  const std::string base = t.dir + "/kernel-" + std::to_string(id) + suffix;
  FILE* man = fopen((base + ".allocs").c_str(), "w");
  if (!man) {
    fprintf(stderr, "asim isa tracer: cannot write %s.allocs\n", base.c_str());
    return;
  }
  fprintf(man, "# alloc_number address bytes file\n");
  size_t total = 0;
  std::vector<uint8_t> buf;
  for (const auto& kv : t.allocs) {
    const auto& a = kv.second;
    std::string fn = "-";
    if (total + a.bytes <= t.snapshot_max) {
      fn = "kernel-" + std::to_string(id) + suffix + "_alloc-" + std::to_string(a.num) + ".bin";
      buf.resize(a.bytes);
      RT_HIP(hipMemcpyDtoH(buf.data(), (hipDeviceptr_t)kv.first, a.bytes));
      FILE* f = fopen((t.dir + "/" + fn).c_str(), "wb");
      if (!f || fwrite(buf.data(), 1, a.bytes, f) != a.bytes) {
        fprintf(stderr, "asim isa tracer: snapshot write failed (%s)\n", fn.c_str());
        exit(3);
      }
      fclose(f);
      total += a.bytes;
    }
    fprintf(man, "%u 0x%016llx %zu %s\n", a.num, (unsigned long long)kv.first, a.bytes, fn.c_str());
  }
  fclose(man);
}

// A kernel's trace could not be captured whole: the capture is unusable, so
// the traced program ends here with a distinct exit status (5) instead of
// leaving a directory whose kernelslist names a partial trace.
[[noreturn]] void fail_run(Tracer& t) {
  FILE* f = fopen((t.dir + "/CAPTURE_FAILED").c_str(), "w");
  if (f) {
    fprintf(f, "trace chunks were lost; this directory is not a complete capture\n");
    fclose(f);
  }
  fflush(stderr);
  _exit(5);
}

Tracer::Ring& ring_for(Tracer& t, int dev) {
  Tracer::Ring& r = t.rings[dev];
  if (r.host) return r;
  const size_t cb = (size_t)kChunkUnits * 16;
  r.slots = 4;  // the probes need a power of two
  while ((size_t)r.slots * 2 * cb <= t.ring_bytes) r.slots *= 2;
  r.shift = (uint32_t)__builtin_ctz(r.slots);
  RT_HIP(hipHostMalloc((void**)&r.host, (size_t)r.slots * cb, hipHostMallocCoherent | hipHostMallocMapped));
  memset(r.host, 0, (size_t)r.slots * cb);
  RT_HIP(hipHostGetDevicePointer((void**)&r.dev, r.host, 0));
  return r;
}

uint32_t tickets_issued(Tracer& t) {
  uint32_t used = 0;
  for (Ctl* sh : t.shadows) {
    Ctl r{};
    RT_HIP(hipMemcpyFromSymbol(&r, (const void*)sh, sizeof(r), 0, hipMemcpyDeviceToHost));
    used = std::max(used, r.next_chunk);
  }
  return used;
}

// the ring path of a traced launch: drain during the kernel, spill, decode
hipError_t launch_streamed(Tracer& t, long id, const std::string& name, const KMap& km,
                           hipError_t (*real)(const void*, dim3, dim3, void**, size_t, hipStream_t), const void* f,
                           dim3 g, dim3 b, void** args, size_t shmem, hipStream_t st, int dev) {
  Tracer::Ring& r = ring_for(t, dev);
  Ctl c{};
  c.buf = (uint64_t)(uintptr_t)r.dev;
  c.n_chunks = r.slots;
  c.mask = r.slots - 1;
  c.shift = r.shift;
  c.spin_limit = t.spin_limit;
  for (Ctl* sh : t.shadows) RT_HIP(hipMemcpyToSymbol((const void*)sh, &c, sizeof(c), 0, hipMemcpyHostToDevice));
  const std::string spath = t.dir + "/.kernel-" + std::to_string(id) + ".chunks";
  Spill sp;
  sp.f = fopen(spath.c_str(), "w+b");
  if (!sp.f) {
    fprintf(stderr, "asim isa tracer: cannot write %s\n", spath.c_str());
    exit(3);
  }
  hipError_t e = real(f, g, b, args, shmem, st);
  if (e != hipSuccess) {
    fclose(sp.f);
    unlink(spath.c_str());
    return e;
  }
  std::atomic<bool> stop{false};
  std::thread drain([&] {
    while (!stop.load(std::memory_order_relaxed)) {
      if (t.drain_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(t.drain_delay_us));
      if (!drain_closed(r, sp)) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  });
  const hipError_t se = hipStreamSynchronize(st);
  stop = true;
  drain.join();
  RT_HIP(se);
  const uint32_t tickets = tickets_issued(t);
  drain_final(r, tickets, sp);
  if (tickets > sp.chunks) {
    // a wave gave up waiting for a ring slot and stopped recording: the
    // trace would be silently truncated, so none is written and the run fails
    // (the reference's channel blocks its producers instead, channel.hpp:56-116;
    // here the wait is bounded so a stalled host cannot hang the GPU)
    fprintf(stderr,
            "asim isa tracer: FATAL: kernel %ld (%s): %u of %u trace chunks lost (a wave waited longer than "
            "ASIM_TRACE_SPIN_LIMIT=%u polls for a ring slot); no trace written for it. Raise ASIM_TRACE_RING_MB "
            "or ASIM_TRACE_SPIN_LIMIT\n",
            id, name.c_str(), tickets - sp.chunks, tickets, t.spin_limit);
    fclose(sp.f);
    unlink(spath.c_str());
    fail_run(t);
  }
  fflush(sp.f);
  const size_t bytes = (size_t)sp.chunks * kChunkUnits * 16;
  const uint8_t* data = nullptr;
  void* m = MAP_FAILED;
  if (bytes) {
    m = mmap(nullptr, bytes, PROT_READ, MAP_PRIVATE, fileno(sp.f), 0);
    if (m == MAP_FAILED) {
      fprintf(stderr, "asim isa tracer: cannot map %s\n", spath.c_str());
      exit(3);
    }
    data = static_cast<const uint8_t*>(m);
  }
  write_kernel(t, id, name, km, g, b, shmem, data, sp.chunks);
  snapshot_allocs(t, id, t.gpu_id >= 0 ? "_" + std::to_string(dev) : "");
  if (m != MAP_FAILED) munmap(m, bytes);
  fclose(sp.f);
  unlink(spath.c_str());
  return e;
}

}  // namespace

extern "C" {

void** __hipRegisterFatBinary(const void* data) {
  using F = void** (*)(const void*);
  static F real = (F)dlsym(RTLD_NEXT, "__hipRegisterFatBinary");
  void** h = real(data);
  Tracer& t = T();
  using RV = void (*)(void**, void*, char*, char*, int, size_t, int, int);
  static RV regvar = (RV)dlsym(RTLD_NEXT, "__hipRegisterVar");
  // the probes' control block: one per code object, registered like a
  // compiler-emitted __device__ variable
  Ctl* shadow = new Ctl();
  static char nm[] = "__asim_tctl";
  regvar(h, shadow, nm, nm, 0, sizeof(Ctl), 0, 0);
  std::lock_guard<std::mutex> g(t.mu);
  t.shadows.push_back(shadow);
  return h;
}

void __hipRegisterFunction(void** modules, const void* hostFunction, char* deviceFunction, const char* deviceName,
                           unsigned int threadLimit, uint3* tid, uint3* bid, dim3* blockDim, dim3* gridDim,
                           int* wSize) {
  using F = void (*)(void**, const void*, char*, const char*, unsigned int, uint3*, uint3*, dim3*, dim3*, int*);
  static F real = (F)dlsym(RTLD_NEXT, "__hipRegisterFunction");
  {
    Tracer& t = T();
    std::lock_guard<std::mutex> g(t.mu);
    t.names[hostFunction] = deviceName ? deviceName : deviceFunction;
  }
  real(modules, hostFunction, deviceFunction, deviceName, threadLimit, tid, bid, blockDim, gridDim, wSize);
}

hipError_t hipMalloc(void** ptr, size_t bytes) {
  using F = hipError_t (*)(void**, size_t);
  static F real = (F)dlsym(RTLD_NEXT, "hipMalloc");
  hipError_t e = real(ptr, bytes);
  Tracer& t = T();
  if (e == hipSuccess && t.enabled && ptr && *ptr) {
    std::lock_guard<std::mutex> g(t.mu);
    t.allocs[(uintptr_t)*ptr] = Tracer::Alloc{t.alloc_count++, bytes};
  }
  return e;
}

hipError_t hipFree(void* ptr) {
  using F = hipError_t (*)(void*);
  static F real = (F)dlsym(RTLD_NEXT, "hipFree");
  Tracer& t = T();
  if (t.enabled && ptr) {
    std::lock_guard<std::mutex> g(t.mu);
    t.allocs.erase((uintptr_t)ptr);
  }
  return real(ptr);
}

hipError_t hipMemcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  using F = hipError_t (*)(void*, const void*, size_t, hipMemcpyKind);
  static F real = (F)dlsym(RTLD_NEXT, "hipMemcpy");
  hipError_t e = real(dst, src, bytes, kind);
  Tracer& t = T();
  if (t.enabled && (kind == hipMemcpyHostToDevice || kind == hipMemcpyDeviceToHost) && t.on_traced_device()) {
    // DtoH copies carry no simulated work but mark a host synchronisation
    // (the next kernel is launched from an idle queue)
    char s[96];
    if (kind == hipMemcpyHostToDevice)
      snprintf(s, sizeof(s), "MemcpyHtoD,0x%016llx,%zu", (unsigned long long)(uintptr_t)dst, bytes);
    else
      snprintf(s, sizeof(s), "MemcpyDtoH,0x%016llx,%zu", (unsigned long long)(uintptr_t)src, bytes);
    std::lock_guard<std::mutex> g(t.mu);
    t.append("kernelslist.g", s);
  }
  return e;
}

hipError_t hipLaunchKernel(const void* f, dim3 g, dim3 b, void** args, size_t shmem, hipStream_t st) {
  using F = hipError_t (*)(const void*, dim3, dim3, void**, size_t, hipStream_t);
  static F real = (F)dlsym(RTLD_NEXT, "hipLaunchKernel");
  Tracer& t = T();
  if (!t.enabled || !t.on_traced_device()) return real(f, g, b, args, shmem, st);
  std::lock_guard<std::mutex> lk(t.mu);
  const long id = ++t.next_id;
  auto nit = t.names.find(f);
  const std::string name = nit == t.names.end() ? "" : nit->second;
  auto mit = t.maps.find(name);
  if (!t.traced(id) || mit == t.maps.end()) {
    if (t.traced(id)) fprintf(stderr, "asim isa tracer: kernel %s has no instrumentation map\n", name.c_str());
    return real(f, g, b, args, shmem, st);
  }
  int dev = 0;
  RT_HIP(hipGetDevice(&dev));
  if (!t.buf_bytes) return launch_streamed(t, id, name, mit->second, real, f, g, b, args, shmem, st, dev);
  Tracer::DevBuf& db = t.bufs[dev];
  if (!db.ptr) {
    // the runtime's own hipMalloc: this interposer's would retake t.mu (held
    // here) and the tracer's buffer is not an application allocation
    using M = hipError_t (*)(void**, size_t);
    static M real_malloc = (M)dlsym(RTLD_NEXT, "hipMalloc");
    RT_HIP(real_malloc((void**)&db.ptr, t.buf_bytes));
    RT_HIP(hipMemset(db.ptr, 0, t.buf_bytes));
  } else if (db.last_used) {
    RT_HIP(hipMemset(db.ptr, 0, (size_t)db.last_used * kChunkUnits * 16));
  }
  Ctl c{};
  c.buf = (uint64_t)(uintptr_t)db.ptr;
  c.n_chunks = (uint32_t)(t.buf_bytes / ((size_t)kChunkUnits * 16));
  for (Ctl* sh : t.shadows) RT_HIP(hipMemcpyToSymbol((const void*)sh, &c, sizeof(c), 0, hipMemcpyHostToDevice));  // the shadow itself, not the template overload (&sh)
  hipError_t e = real(f, g, b, args, shmem, st);
  if (e != hipSuccess) return e;
  RT_HIP(hipStreamSynchronize(st));
  uint32_t used = tickets_issued(t);
  db.last_used = std::min(used, c.n_chunks);
  if (used > c.n_chunks) {
    // the waves past the end stopped recording: no usable trace of this kernel
    fprintf(stderr,
            "asim isa tracer: FATAL: kernel %ld (%s) needs %u chunks of %u KB, the device buffer holds %u: no trace "
            "written (unset ASIM_TRACE_BUF_MB to stream through the host ring)\n",
            id, name.c_str(), used, kChunkUnits / 64, c.n_chunks);
    fail_run(t);
  }
  std::vector<uint8_t> host((size_t)used * kChunkUnits * 16);
  // the tracer's own read-back is not an application copy (no trace line)
  if (used) RT_HIP(hipMemcpyDtoH(host.data(), db.ptr, host.size()));
  write_kernel(t, id, name, mit->second, g, b, shmem, host.data(), used);
  snapshot_allocs(t, id, t.gpu_id >= 0 ? "_" + std::to_string(dev) : "");
  return e;
}

}  // extern "C"
