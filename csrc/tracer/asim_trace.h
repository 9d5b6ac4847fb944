// Device-side trace capture for HIP applications on MI355X (wave64).
//
// The reference captures SASS traces by binary instrumentation (NVBit,
// util/tracer_nvbit/tracer_tool/inject_funcs.cu:20-81 ballots the active and
// predicate masks, shuffles 32 lane addresses and pushes a record into a
// device->host channel, channel.hpp:56-116).  CDNA4 has no binary
// instrumentation framework in this stack, so the same information is
// captured at the source level: a kernel is written once as a template over
// a trace policy (the single-source idiom of this framework's cycle model)
//
//     template <class TR> __global__ void k(TR tr, ...) {
//       auto w = tr.wave();                                   // per-wave context
//       ASIM_VALU(w, asim_trace::V_MAD_U32_U24, 1, 0, 0);    // dst, src, src
//       if (i < n) {
//         float x = ASIM_LD(w, asim_trace::GLOBAL_LOAD_DWORD, a + i, 2, 1);
//         ASIM_ST(w, asim_trace::GLOBAL_STORE_DWORD, c + i, x, 2, 1);
//       }
//       w.exit();
//     }
//
// and launched with asim_trace::launch(name, k<On>, k<Off>, ...).  With
// ASIM_TRACE_DIR unset the Off instantiation runs (every hook compiles to the
// plain operation); with it set the On instantiation runs on the GPU and each
// wave's leader lane pushes 32-byte records (64-bit exec mask from __ballot,
// CDNA opcode, register ids, per-wave sequence number) into a device buffer,
// every active lane writing its own address for memory operations.  The host
// then writes kernel-N.traceg (trace format v4, wavefront size 64, binary
// version 950) plus kernelslist.g, ready for the simulator or for
// conversion to the binary .asimk format.
#pragma once
#include <filesystem>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace asim_trace {

// CDNA4 opcodes the annotations use (names are the ISA mnemonics)
enum Op : uint16_t {
  V_ADD_F32 = 0, V_MUL_F32, V_FMA_F32, V_ADD_F64, V_MUL_F64, V_FMA_F64, V_ADD_U32, V_MAD_U32_U24, V_MUL_LO_U32,
  V_LSHLREV_B32, V_AND_B32, V_CMP_GT_I32, V_CNDMASK_B32, V_MAX_F32, V_MIN_F32, V_EXP_F32, V_LOG_F32, V_SQRT_F32,
  V_RCP_F32, S_ADD_U32, S_MUL_I32, S_CMP_LT_I32, S_CBRANCH_SCC1, S_BRANCH, S_WAITCNT, S_BARRIER, S_ENDPGM,
  GLOBAL_LOAD_DWORD, GLOBAL_LOAD_DWORDX2, GLOBAL_LOAD_DWORDX4, GLOBAL_STORE_DWORD, GLOBAL_STORE_DWORDX2,
  GLOBAL_STORE_DWORDX4, GLOBAL_ATOMIC_ADD, DS_READ_B32, DS_READ_B64, DS_WRITE_B32, DS_WRITE_B64,
  V_MFMA_F32_32X32X16_BF16, OP_COUNT
};

inline const char* op_name(uint16_t op) {
  static const char* const names[OP_COUNT] = {
      "v_add_f32", "v_mul_f32", "v_fma_f32", "v_add_f64", "v_mul_f64", "v_fma_f64", "v_add_u32", "v_mad_u32_u24",
      "v_mul_lo_u32", "v_lshlrev_b32", "v_and_b32", "v_cmp_gt_i32", "v_cndmask_b32", "v_max_f32", "v_min_f32",
      "v_exp_f32", "v_log_f32", "v_sqrt_f32", "v_rcp_f32", "s_add_u32", "s_mul_i32", "s_cmp_lt_i32",
      "s_cbranch_scc1", "s_branch", "s_waitcnt", "s_barrier", "s_endpgm", "global_load_dword",
      "global_load_dwordx2", "global_load_dwordx4", "global_store_dword", "global_store_dwordx2",
      "global_store_dwordx4", "global_atomic_add", "ds_read_b32", "ds_read_b64", "ds_write_b32", "ds_write_b64",
      "v_mfma_f32_32x32x16_bf16"};
  return op < OP_COUNT ? names[op] : "s_nop";
}

inline int op_width(uint16_t op) {
  switch (op) {
    case GLOBAL_LOAD_DWORDX2: case GLOBAL_STORE_DWORDX2: case DS_READ_B64: case DS_WRITE_B64: return 8;
    case GLOBAL_LOAD_DWORDX4: case GLOBAL_STORE_DWORDX4: return 16;
    case GLOBAL_LOAD_DWORD: case GLOBAL_STORE_DWORD: case GLOBAL_ATOMIC_ADD: case DS_READ_B32: case DS_WRITE_B32:
      return 4;
    default: return 0;
  }
}

__host__ __device__ inline bool op_is_lds(uint16_t op) { return op >= DS_READ_B32 && op <= DS_WRITE_B64; }

// one wave-level instruction (32 bytes)
struct Rec {
  uint64_t mask;
  uint32_t cta;       // linear CTA id
  uint32_t addr_row;  // row of 64 addresses, or ~0u
  uint32_t seq;       // per-wave program order
  uint16_t warp;      // wave index within the CTA
  uint16_t op;
  uint8_t dst, src0, src1, src2;
  uint32_t pc;
};
static_assert(sizeof(Rec) == 32, "Rec layout");

struct Channel {
  Rec* recs = nullptr;
  uint64_t* addrs = nullptr;                   // rows of 64
  unsigned long long* counters = nullptr;      // [0] records [1] address rows
  unsigned long long cap_recs = 0, cap_rows = 0;
};

// ------------------------------------------------------------------ policies
struct OffWave {
  __device__ void valu(uint32_t, uint16_t, uint8_t, uint8_t, uint8_t = 0, uint8_t = 0) {}
  template <class T>
  __device__ T ld(uint32_t, uint16_t, const T* p, uint8_t, uint8_t) {
    return *p;
  }
  template <class T>
  __device__ void st(uint32_t, uint16_t, T* p, T v, uint8_t, uint8_t) {
    *p = v;
  }
  template <class T>
  __device__ T atomic_add(uint32_t, T* p, T v, uint8_t, uint8_t) {
    return atomicAdd(p, v);
  }
  __device__ void barrier(uint32_t) { __syncthreads(); }
  __device__ void exit(uint32_t = 0) {}
};

struct Off {
  __device__ OffWave wave() const { return OffWave{}; }
};

struct OnWave {
  Channel ch;
  uint32_t cta;
  uint16_t warp;
  uint32_t* seq;  // LDS counter of this wave

  __device__ void emit(uint32_t pc, uint16_t op, uint8_t dst, uint8_t s0, uint8_t s1, uint8_t s2, const void* addr) {
    const uint64_t mask = __ballot(1);
    const int leader = __ffsll((unsigned long long)mask) - 1;
    const int lane = (int)__lane_id();
    unsigned long long slot = 0, row = ~0ull;
    if (lane == leader) {
      slot = atomicAdd(&ch.counters[0], 1ull);
      if (addr) row = atomicAdd(&ch.counters[1], 1ull);
    }
    slot = __shfl(slot, leader);
    row = __shfl(row, leader);
    if (addr && row < ch.cap_rows) {
      uint64_t a = (uint64_t)(uintptr_t)addr;
      if (op_is_lds(op)) a &= 0xffffffffull;  // LDS offset inside the shared aperture
      ch.addrs[row * 64 + lane] = a;
    }
    if (lane == leader) {
      const uint32_t s = (*seq)++;
      if (slot < ch.cap_recs) {
        Rec r;
        r.mask = mask;
        r.cta = cta;
        r.addr_row = addr && row < ch.cap_rows ? (uint32_t)row : ~0u;
        r.seq = s;
        r.warp = warp;
        r.op = op;
        r.dst = dst;
        r.src0 = s0;
        r.src1 = s1;
        r.src2 = s2;
        r.pc = pc;
        ch.recs[slot] = r;
      }
    }
  }
  __device__ void valu(uint32_t pc, uint16_t op, uint8_t dst, uint8_t s0, uint8_t s1 = 0, uint8_t s2 = 0) {
    emit(pc, op, dst, s0, s1, s2, nullptr);
  }
  template <class T>
  __device__ T ld(uint32_t pc, uint16_t op, const T* p, uint8_t dst, uint8_t areg) {
    emit(pc, op, dst, areg, 0, 0, p);
    return *p;
  }
  template <class T>
  __device__ void st(uint32_t pc, uint16_t op, T* p, T v, uint8_t vreg, uint8_t areg) {
    emit(pc, op, 0, areg, vreg, 0, p);
    *p = v;
  }
  template <class T>
  __device__ T atomic_add(uint32_t pc, T* p, T v, uint8_t dst, uint8_t areg) {
    emit(pc, GLOBAL_ATOMIC_ADD, dst, areg, 0, 0, p);
    return atomicAdd(p, v);
  }
  __device__ void barrier(uint32_t pc) {
    emit(pc, S_BARRIER, 0, 0, 0, 0, nullptr);
    __syncthreads();
  }
  __device__ void exit(uint32_t pc = 0xfffff) { emit(pc, S_ENDPGM, 0, 0, 0, 0, nullptr); }
};

struct On {
  Channel ch;
  __device__ OnWave wave() const {
    __shared__ uint32_t seq[32];  // one counter per wave of the CTA (<= 2048 threads)
    const uint32_t tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
    const uint16_t w = (uint16_t)(tid / 64);
    if ((tid & 63) == 0) seq[w] = 0;
    OnWave o;
    o.ch = ch;
    o.cta = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    o.warp = w;
    o.seq = &seq[w];
    return o;
  }
};

// call-site PCs: 8 bytes per source line keeps distinct sites distinct
#define ASIM_PC ((uint32_t)(__LINE__ * 8))
#define ASIM_VALU(w, op, ...) (w).valu(ASIM_PC, op, __VA_ARGS__)
#define ASIM_LD(w, op, p, dst, areg) (w).ld(ASIM_PC, op, p, dst, areg)
#define ASIM_ST(w, op, p, v, vreg, areg) (w).st(ASIM_PC, op, p, v, vreg, areg)
#define ASIM_ATOMIC_ADD(w, p, v, dst, areg) (w).atomic_add(ASIM_PC, p, v, dst, areg)
#define ASIM_BARRIER(w) (w).barrier(ASIM_PC)

// --------------------------------------------------------------------- host
#define ASIM_HIP(x)                                                                                         \
  do {                                                                                                      \
    hipError_t e_ = (x);                                                                                    \
    if (e_ != hipSuccess) {                                                                                 \
      fprintf(stderr, "asim_trace: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);  \
      exit(3);                                                                                              \
    }                                                                                                       \
  } while (0)

struct Session {
  std::string dir;
  int next_id = 1;
  bool enabled = false;
  int kstart = 0, kend = 1 << 30;  // kernel-range tracing (reference DYNAMIC_KERNEL_LIMIT_START/END)
  unsigned long long cap_recs = 8ull << 20, cap_rows = 1ull << 20;
  Session() {
    const char* d = getenv("ASIM_TRACE_DIR");
    if (d && *d) {
      dir = d;
      enabled = true;
      {
        std::error_code ec;
        std::filesystem::create_directories(dir, ec);
        if (ec) fprintf(stderr, "asim_trace: cannot create %s\n", d);
      }
      FILE* f = fopen((dir + "/kernelslist.g").c_str(), "w");
      if (f) fclose(f);
      f = fopen((dir + "/stats.csv").c_str(), "w");
      if (f) {
        fprintf(f, "kernel id, kernel name, grid_dim, block_dim, #warp insts, #thread insts\n");
        fclose(f);
      }
    }
    if (const char* s = getenv("ASIM_TRACE_KERNEL_START")) kstart = atoi(s);
    if (const char* s = getenv("ASIM_TRACE_KERNEL_END")) kend = atoi(s);
    if (const char* s = getenv("ASIM_TRACE_MAX_RECORDS")) cap_recs = strtoull(s, nullptr, 0);
    if (const char* s = getenv("ASIM_TRACE_MAX_MEMOPS")) cap_rows = strtoull(s, nullptr, 0);
  }
  static Session& get() {
    static Session s;
    return s;
  }
  void append_list(const std::string& line) {
    if (!enabled) return;
    FILE* f = fopen((dir + "/kernelslist.g").c_str(), "a");
    if (f) {
      fprintf(f, "%s\n", line.c_str());
      fclose(f);
    }
  }
};

inline void memcpy_htod(void* dst, const void* src, size_t bytes) {
  ASIM_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  char buf[96];
  snprintf(buf, sizeof(buf), "MemcpyHtoD,0x%016llx,%zu", (unsigned long long)(uintptr_t)dst, bytes);
  Session::get().append_list(buf);
}

inline void write_trace(const std::string& path, const char* name, int id, dim3 g, dim3 b, size_t shmem,
                        std::vector<Rec>& recs, const std::vector<uint64_t>& addrs, uint64_t* thread_insts) {
  std::sort(recs.begin(), recs.end(), [](const Rec& x, const Rec& y) {
    if (x.cta != y.cta) return x.cta < y.cta;
    if (x.warp != y.warp) return x.warp < y.warp;
    return x.seq < y.seq;
  });
  FILE* f = fopen(path.c_str(), "w");
  if (!f) {
    fprintf(stderr, "asim_trace: cannot write %s\n", path.c_str());
    exit(3);
  }
  fprintf(f, "-kernel name = %s\n-kernel id = %d\n-grid dim = (%u,%u,%u)\n-block dim = (%u,%u,%u)\n-shmem = %zu\n",
          name, id, g.x, g.y, g.z, b.x, b.y, b.z, shmem);
  fprintf(f, "-nregs = 32\n-binary version = 950\n-wavefront size = 64\n-hip stream id = 0\n");
  fprintf(f, "-shmem base_addr = 0x0\n-local mem base_addr = 0x0\n-rocprofiler version = asim_trace\n");
  fprintf(f, "-accelsim tracer version = 4\n\n");
  fprintf(f, "#traces format = PC mask dest_num reg_dests opcode src_num reg_srcs mem_width mem_addresses\n\n");
  uint64_t ti = 0;
  size_t i = 0;
  while (i < recs.size()) {
    const uint32_t cta = recs[i].cta;
    const uint32_t x = cta % g.x, y = (cta / g.x) % g.y, z = cta / (g.x * g.y);
    fprintf(f, "#BEGIN_TB\n\nthread block = %u,%u,%u\n\n", x, y, z);
    while (i < recs.size() && recs[i].cta == cta) {
      const uint16_t w = recs[i].warp;
      size_t j = i;
      while (j < recs.size() && recs[j].cta == cta && recs[j].warp == w) ++j;
      fprintf(f, "warp = %u\ninsts = %zu\n", w, j - i);
      for (size_t k = i; k < j; ++k) {
        const Rec& r = recs[k];
        ti += (uint64_t)__builtin_popcountll(r.mask);
        fprintf(f, "%04x %016llx ", r.pc, (unsigned long long)r.mask);
        if (r.dst) fprintf(f, "1 v%u ", r.dst - 1);
        else fprintf(f, "0 ");
        const uint8_t src[3] = {r.src0, r.src1, r.src2};
        int ns = 0;
        for (int q = 0; q < 3; ++q) ns += src[q] != 0;
        fprintf(f, "%s %d", op_name(r.op), ns);
        for (int q = 0; q < 3; ++q)
          if (src[q]) fprintf(f, " v%u", src[q] - 1);
        const int width = op_width(r.op);
        if (width && r.addr_row != ~0u) {
          fprintf(f, " %d 0", width);
          for (int l = 0; l < 64; ++l)
            if ((r.mask >> l) & 1ull) fprintf(f, " 0x%llx", (unsigned long long)addrs[(size_t)r.addr_row * 64 + l]);
        } else {
          fprintf(f, " 0");
        }
        fprintf(f, "\n");
      }
      i = j;
    }
    fprintf(f, "\n#END_TB\n\n");
  }
  fclose(f);
  *thread_insts = ti;
}

// Launch `traced` (tracing on and the kernel inside the traced range) or
// `plain`; both instantiations take the policy as the first argument.
template <class... KArgs, class... Args>
void launch(const char* name, void (*traced)(On, KArgs...), void (*plain)(Off, KArgs...), dim3 g, dim3 b,
            size_t shmem, hipStream_t st, Args... args) {
  Session& s = Session::get();
  const int id = s.next_id++;
  if (!s.enabled || id < s.kstart || id > s.kend) {
    hipLaunchKernelGGL(plain, g, b, shmem, st, Off{}, args...);
    ASIM_HIP(hipGetLastError());
    return;
  }
  On on;
  ASIM_HIP(hipMalloc(&on.ch.recs, s.cap_recs * sizeof(Rec)));
  ASIM_HIP(hipMalloc(&on.ch.addrs, s.cap_rows * 64 * sizeof(uint64_t)));
  ASIM_HIP(hipMalloc(&on.ch.counters, 2 * sizeof(unsigned long long)));
  ASIM_HIP(hipMemset(on.ch.counters, 0, 2 * sizeof(unsigned long long)));
  on.ch.cap_recs = s.cap_recs;
  on.ch.cap_rows = s.cap_rows;
  hipLaunchKernelGGL(traced, g, b, shmem, st, on, args...);
  ASIM_HIP(hipGetLastError());
  ASIM_HIP(hipStreamSynchronize(st));
  unsigned long long cnt[2];
  ASIM_HIP(hipMemcpy(cnt, on.ch.counters, sizeof(cnt), hipMemcpyDeviceToHost));
  if (cnt[0] > s.cap_recs || cnt[1] > s.cap_rows) {
    fprintf(stderr, "asim_trace: kernel %s overflowed the trace buffers (%llu records, %llu memops); raise "
                    "ASIM_TRACE_MAX_RECORDS / ASIM_TRACE_MAX_MEMOPS\n", name, cnt[0], cnt[1]);
    exit(4);
  }
  std::vector<Rec> recs(cnt[0]);
  std::vector<uint64_t> addrs(cnt[1] * 64);
  if (cnt[0]) ASIM_HIP(hipMemcpy(recs.data(), on.ch.recs, cnt[0] * sizeof(Rec), hipMemcpyDeviceToHost));
  if (cnt[1]) ASIM_HIP(hipMemcpy(addrs.data(), on.ch.addrs, cnt[1] * 64 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  ASIM_HIP(hipFree(on.ch.recs));
  ASIM_HIP(hipFree(on.ch.addrs));
  ASIM_HIP(hipFree(on.ch.counters));
  const std::string fn = "kernel-" + std::to_string(id) + ".traceg";
  uint64_t ti = 0;
  write_trace(s.dir + "/" + fn, name, id, g, b, shmem, recs, addrs, &ti);
  s.append_list(fn);
  FILE* f = fopen((s.dir + "/stats.csv").c_str(), "a");
  if (f) {
    fprintf(f, "kernel-%d, %s, (%u,%u,%u), (%u,%u,%u), %zu, %llu\n", id, name, g.x, g.y, g.z, b.x, b.y, b.z,
            recs.size(), (unsigned long long)ti);
    fclose(f);
  }
}

}  // namespace asim_trace
