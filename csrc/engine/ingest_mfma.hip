// Trace ingest on the MI355X matrix cores.
//
// Every memory instruction of a kernel trace is reduced at ingest to what the
// cycle model consumes (reference: the per-warp access generation of
// abstract_hardware_model.cc:475-586 and the shared-memory bank-conflict count
// of shader.cc / gpu-cache bank hashing):
//   * shared-memory instructions -> the bank-conflict degree: per part of the
//     warp, the largest number of DISTINCT 4-byte words that fall into one
//     bank;
//   * global / local instructions -> the ascending list of 128 B lines they
//     touch, each with its 32 B sector mask and byte count.
// Both are occupancy matrices, computed here as one-hot products on
// v_mfma_f32_32x32x16_bf16 (0/1 and small-integer operands are exact in bf16,
// the f32 accumulations exact below 2^24):
//   * O[row][bank] = sum over (lane, word) slots of onehot(row) x onehot(bank)
//     with row = word / n_banks relative to the instruction's lowest row; the
//     distinct words of a bank are the non-zero rows of its column, so the
//     degree is max over banks of nnz(column) -- the accumulator keeps the
//     column on the lane (C/D: col = lane & 31), nnz is a per-lane count plus
//     one cross-half add;
//   * Q[q][line] = sum over (lane, piece) slots of value_q(slot) x
//     onehot(line) with q = sector 0..3 touched, 4 = bytes, line relative to
//     the lowest line: rows 0..3 land in registers 0..3 of lanes 0..31 and
//     row 4 in register 0 of lanes 32..63; a line is touched when any sector
//     count is non-zero, and the columns come out in ascending line order, so
//     a ballot prefix gives each line its output index.
// One wavefront per instruction, four per workgroup, slots staged in LDS.
// Instructions outside the windows (rows spanning > 256, lines spanning > 64,
// > 8 words or > 2 lines per lane, limited-broadcast or non-32/64-bank
// configurations) are flagged and coalesced on the host with the same code as
// the CPU path (trace.cc coalesce_lanes / smem_conflict_degree), so the result
// is bit-identical to coalesce_kernel (tests/test_ingest_mfma.py).
#include <hip/hip_runtime.h>

#include <chrono>
#include <stdexcept>
#include <string>
#include <vector>

#include "../trace/trace.h"

namespace asim {

#define IHIPCHECK(x)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr uint32_t kFallback = 0xffffffffu;
constexpr uint32_t kNoSlot = 0xffffffffu;
constexpr int kWavesPerGroup = 4;
constexpr int kSlots = 64 * 8;      // per-wave LDS slots: 64 lanes x 8 words (or 2 line pieces)
constexpr uint32_t kRowTiles = 8;   // bank-conflict window: 8 x 32 rows
constexpr uint32_t kLineTiles = 2;  // coalescer window: 2 x 32 lines (= kMaxAccess)
static_assert(kLineTiles * 32 == (uint32_t)kMaxAccess, "the line window is the access cap");

struct IngJob {
  uint64_t mask;
  uint64_t base;
  int32_t stride;
  uint32_t list;
  uint16_t width;
  uint8_t kind;
  uint8_t pad0;
  uint32_t pad1;
};
static_assert(sizeof(IngJob) == 32, "IngJob is 32 bytes");

constexpr int kMaxGroupTables = 8;
struct IngGroups {
  uint32_t n, nb;
  uint64_t lanes[8];
};
struct IngParams {
  uint32_t ws, nb, parts, l1_banks;
  IngGroups groups[kMaxGroupTables];  // CDNA4 lane-group tables (IngJob::pad0 - 1)
};

__device__ __forceinline__ uint64_t wmin64(uint64_t v) {
  for (int o = 32; o; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wmax64(uint64_t v) {
  for (int o = 32; o; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wmax32(uint32_t v) {
  for (int o = 32; o; o >>= 1) {
    const uint32_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// small non-negative integer -> bf16 (exact up to 256: the low 16 bits of the
// f32 pattern are zero)
__device__ __forceinline__ __bf16 bf(uint32_t v) {
  return __builtin_bit_cast(__bf16, (unsigned short)(__builtin_bit_cast(uint32_t, (float)v) >> 16));
}

// distinct words of the busiest bank over the lanes with `pa` set
// (trace.cc lanes_degree): 0 without such lanes, kFallback outside the windows
__device__ uint32_t group_degree(bool pa, uint64_t w0, uint64_t w1, uint32_t nw, uint32_t nb, uint32_t* sl,
                                 uint32_t& nmfma) {
  const int l = (int)(threadIdx.x & 63);
  if (!__ballot(pa)) return 0;
  const uint32_t nwmax = wmax32(pa ? nw : 0u);
  if (nwmax > 8) return kFallback;
  const uint64_t rlo = wmin64(pa ? w0 / nb : ~0ull);
  const uint64_t rhi = wmax64(pa ? w1 / nb : 0ull);
  if (rhi - rlo >= 32ull * kRowTiles) return kFallback;
  const uint32_t ntr = (uint32_t)((rhi - rlo) / 32) + 1;
  for (uint32_t j = 0; j < nwmax; ++j) {
    const uint64_t w = w0 + j;
    sl[j * 64 + l] = (pa && j < nw) ? ((uint32_t)(w / nb - rlo) << 8 | (uint32_t)(w % nb)) : kNoSlot;
  }
  wave_sync();
  const uint32_t ksteps = nwmax * 4;  // 64 slots per word index, 16 per MFMA
  const uint32_t h = (uint32_t)l >> 5, c32 = (uint32_t)l & 31;
  uint32_t deg = 0;
  for (uint32_t ct = 0; ct < nb / 32; ++ct) {
    uint32_t cnt = 0;
    for (uint32_t rt = 0; rt < ntr; ++rt) {
      f32x16 acc = {};
      for (uint32_t ks = 0; ks < ksteps; ++ks) {
        bf16x8 a, b;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t v = sl[ks * 16 + 8 * h + e];
          const bool valid = v != kNoSlot;
          a[e] = bf(valid && (v >> 8) == rt * 32 + c32 ? 1u : 0u);   // A[row c32][k]
          b[e] = bf(valid && (v & 0xffu) == ct * 32 + c32 ? 1u : 0u);  // B[k][bank c32]
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        ++nmfma;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) cnt += acc[r] != 0.0f ? 1u : 0u;
    }
    cnt += __shfl_xor(cnt, 32);  // both halves hold rows of the same bank column
    deg = max(deg, wmax32(cnt));
  }
  wave_sync();
  return deg;
}

// conflict degree of one shared-memory instruction (trace.cc smem_conflict_degree)
__device__ uint32_t smem_degree(const IngJob& jb, bool act, uint64_t addr, const IngParams& p, uint32_t* sl,
                                uint32_t& nmfma) {
  const int l = (int)(threadIdx.x & 63);
  const uint64_t wb = jb.width ? jb.width : 4;
  const uint64_t w0 = addr >> 2, w1 = (addr + wb - 1) >> 2;
  const uint32_t nw = act ? (uint32_t)(w1 - w0 + 1) : 0u;
  if (jb.pad0) {
    // CDNA4 lane groups: 1 + the extra cycles over the groups
    const IngGroups& g = p.groups[jb.pad0 - 1];
    uint32_t extra = 0;
    for (uint32_t i = 0; i < g.n; ++i) {
      const uint32_t d = group_degree(act && ((g.lanes[i] >> l) & 1ull), w0, w1, nw, g.nb, sl, nmfma);
      if (d == kFallback) return kFallback;
      extra += d > 1 ? d - 1 : 0;
    }
    return 1 + extra;
  }
  const uint32_t per = (p.ws + p.parts - 1) / p.parts;
  uint32_t total = 0;
  for (uint32_t part = 0; part < p.parts; ++part) {
    const bool inpart = (uint32_t)l >= part * per && (uint32_t)l < (part + 1) * per && (uint32_t)l < p.ws;
    const uint32_t deg = group_degree(act && inpart, w0, w1, nw, p.nb, sl, nmfma);
    if (deg == kFallback) return kFallback;
    total += deg ? deg : (part == 0 ? 1u : 0u);
  }
  return total ? total : 1u;
}

// sorted line accesses of one global instruction (trace.cc coalesce_lanes);
// returns the count, entries written at out[0..n)
__device__ uint32_t gmem_lines(const IngJob& jb, bool act, uint64_t addr, const IngParams& p, uint32_t* sl,
                               TAcc* outbase, uint32_t* cursor, uint32_t* off_out, uint32_t& nmfma) {
  const int l = (int)(threadIdx.x & 63);
  const uint64_t width = jb.width ? jb.width : 4;
  const uint64_t end = addr + width;
  const uint32_t np = act ? (uint32_t)(((end - 1) >> 7) - (addr >> 7) + 1) : 0u;
  const uint32_t npmax = wmax32(np);
  if (npmax > 2) return kFallback;
  if (npmax == 0) {
    if (l == 0) *off_out = 0;
    return 0;
  }
  const uint64_t lmin = wmin64(act ? (addr & ~127ull) : ~0ull);
  const uint64_t lmax = wmax64(act ? ((end - 1) & ~127ull) : 0ull);
  if ((lmax - lmin) / 128 >= 32ull * kLineTiles) return kFallback;
  for (uint32_t j = 0; j < npmax; ++j) {
    uint32_t v = kNoSlot;
    if (j < np) {
      const uint64_t line = (addr & ~127ull) + 128ull * j;
      const uint64_t a = j == 0 ? addr : line;
      const uint64_t pend = end < line + 128 ? end : line + 128;
      uint32_t sec = 0;
      for (uint64_t s = a >> 5; s <= (pend - 1) >> 5; ++s) sec |= 1u << (s & 3);
      v = (uint32_t)((line - lmin) >> 7) | sec << 8 | (uint32_t)(pend - a) << 16;
    }
    sl[j * 64 + l] = v;
  }
  wave_sync();
  const uint32_t ksteps = npmax * 4;
  const uint32_t h = (uint32_t)l >> 5, c32 = (uint32_t)l & 31;
  const uint32_t ntl = (uint32_t)((lmax - lmin) / 128 / 32) + 1;
  uint32_t present[kLineTiles] = {}, secs[kLineTiles] = {}, bytes[kLineTiles] = {};
  for (uint32_t ct = 0; ct < ntl; ++ct) {
    f32x16 acc = {};
    for (uint32_t ks = 0; ks < ksteps; ++ks) {
      bf16x8 a, b;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t v = sl[ks * 16 + 8 * h + e];
        const bool valid = v != kNoSlot;
        // A[q = c32][k]: sector q touched (q < 4), bytes (q == 4)
        const uint32_t q = c32;
        const uint32_t av = !valid ? 0u : q < 4 ? ((v >> (8 + q)) & 1u) : q == 4 ? (v >> 16) : 0u;
        a[e] = bf(av);
        b[e] = bf(valid && (v & 0xffu) == ct * 32 + c32 ? 1u : 0u);  // B[k][line c32]
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      ++nmfma;
    }
    // C/D: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5):
    // lanes 0..31 hold rows 0..3 (sector counts) in registers 0..3, lanes
    // 32..63 row 4 (bytes) in register 0
    const uint32_t by = (uint32_t)__shfl((int)acc[0], (int)(c32 + 32));
    uint32_t sm = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) sm |= acc[q] != 0.0f ? 1u << q : 0u;
    present[ct] = h == 0 && sm != 0;
    secs[ct] = sm;
    bytes[ct] = by;
  }
  wave_sync();
  uint32_t n = 0;
  for (uint32_t ct = 0; ct < ntl; ++ct) n += (uint32_t)__popcll((uint64_t)__ballot(present[ct]));
  uint32_t off = 0;
  if (l == 0) off = atomicAdd(cursor, n);
  off = (uint32_t)__shfl((int)off, 0);
  if (l == 0) *off_out = off;
  const uint64_t below = (1ull << l) - 1ull;
  uint32_t base = 0;
  for (uint32_t ct = 0; ct < ntl; ++ct) {
    const uint64_t m = (uint64_t)__ballot(present[ct]);
    if (present[ct]) {
      const uint32_t idx = base + (uint32_t)__popcll(m & below);
      TAcc t{};
      t.line = lmin + 128ull * (ct * 32 + c32);
      t.sectors = (uint8_t)secs[ct];
      t.bytes = (uint16_t)(bytes[ct] < 128 ? bytes[ct] : 128);
      t.bank = (uint8_t)((t.line >> 7) % (p.l1_banks ? p.l1_banks : 1u));
      t.pad = 0;
      outbase[off + idx] = t;
    }
    base += (uint32_t)__popcll(m);
  }
  return n;
}

__global__ void __launch_bounds__(64 * kWavesPerGroup)
    ingest_kernel(const IngJob* __restrict__ jobs, uint32_t njobs, const uint64_t* __restrict__ addrs, IngParams p,
                  uint32_t* res, uint32_t* offs, uint32_t* nmf, TAcc* accs, uint32_t* cursor) {
  __shared__ uint32_t slots[kWavesPerGroup][kSlots];
  const int w = (int)(threadIdx.x >> 6), l = (int)(threadIdx.x & 63);
  const uint32_t j = blockIdx.x * kWavesPerGroup + (uint32_t)w;
  if (j >= njobs) return;  // whole wavefront: no workgroup barrier below
  const IngJob jb = jobs[j];
  const bool act = (uint32_t)l < p.ws && ((jb.mask >> l) & 1ull);
  uint64_t addr = 0;
  if (act) {
    const uint32_t rank = (uint32_t)__popcll(jb.mask & ((1ull << l) - 1ull));
    addr = jb.list == kNoMem ? jb.base + (uint64_t)((int64_t)jb.stride * (int64_t)rank) : addrs[jb.list + rank];
  }
  uint32_t nmfma = 0;
  uint32_t r;
  if (jb.kind == IK_SMEM)
    r = smem_degree(jb, act, addr, p, slots[w], nmfma);
  else
    r = gmem_lines(jb, act, addr, p, slots[w], accs, cursor, offs + j, nmfma);
  if (l == 0) {
    res[j] = r;
    nmf[j] = nmfma;
  }
}

// device buffers and stream of one host thread, grown on demand and kept
// across kernels (a simulation ingests every kernel of a trace from the
// same one or two threads: the driver and its prefetch thread)
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    n = n ? n : 16;
    if (p && cap >= n) return;
    if (p) IHIPCHECK(hipFree(p));
    p = nullptr;
    cap = 0;
    IHIPCHECK(hipMalloc(&p, n + n / 4));
    cap = n + n / 4;
  }
  template <class T>
  T* get() const {
    return static_cast<T*>(p);
  }
};
struct IngestCtx {
  int device = -1;
  hipStream_t stream = nullptr;
  DevBuf addrs, jobs, res, offs, nmf, acc, cur;
  uint32_t* h_cur = nullptr;  // pinned
  ~IngestCtx() { release(); }
  void release() {
    for (DevBuf* b : {&addrs, &jobs, &res, &offs, &nmf, &acc, &cur}) {
      if (b->p) (void)hipFree(b->p);
      b->p = nullptr;
      b->cap = 0;
    }
    if (h_cur) (void)hipHostFree(h_cur);
    if (stream) (void)hipStreamDestroy(stream);
    h_cur = nullptr;
    stream = nullptr;
  }
  void bind(int dev) {
    if (device == dev && stream) return;
    release();
    device = dev;
    IHIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    IHIPCHECK(hipHostMalloc(&h_cur, 4));
  }
};
IngestCtx& ctx() {
  static thread_local IngestCtx c;
  return c;
}

}  // namespace

bool gpu_coalesce_kernel(const HostKernel& k, const SimCfg& c, int device, ReadyKernel& r, IngestStats* st) {
  int ndev = 0;
  if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return false;
  const auto t0 = std::chrono::steady_clock::now();
  int cur = -1;
  IHIPCHECK(hipGetDevice(&cur));
  // the calling thread's device is restored however this returns
  struct DeviceGuard {
    int prev, now;
    ~DeviceGuard() {
      if (prev != now) (void)hipSetDevice(prev);
    }
  } guard{cur, device};
  if (cur != device) IHIPCHECK(hipSetDevice(device));
  const uint32_t ws = k.h.warp_size ? k.h.warp_size : 32;
  if (ws > 64) return false;
  r = ingest_shell(k);
  const uint64_t name_hash = std::hash<std::string>{}(k.h.name);
  const uint32_t nb = c.smem_banks ? c.smem_banks : 32;
  const uint32_t parts = c.smem_warp_parts ? c.smem_warp_parts : 1;
  const bool smem_dev = !c.smem_limited_bcast && (nb == 32 || nb == 64) && parts <= ws;
  IngParams prm{};
  prm.ws = ws;
  prm.nb = nb;
  prm.parts = parts;
  prm.l1_banks = c.l1_banks;
  std::vector<const LdsGroups*> tabs;  // distinct lane-group tables of this kernel
  const size_t n = r.insts.size();
  std::vector<uint8_t> kind(n);
  std::vector<uint32_t> job_of(n, kNoMem);
  std::vector<IngJob> jobs;
  for (size_t i = 0; i < n; ++i) {
    TInst& in = r.insts[i];
    kind[i] = ingest_prepare(in, c);
    const LdsGroups* lg = kind[i] == IK_SMEM ? lds_groups(c, in.opcode, ws) : nullptr;
    uint32_t tab = 0;
    if (lg) {
      size_t t = 0;
      while (t < tabs.size() && tabs[t] != lg) ++t;
      if (t == tabs.size() && t < (size_t)kMaxGroupTables) {
        tabs.push_back(lg);
        IngGroups& G = prm.groups[t];
        G.n = lg->n;
        G.nb = lg->nb;
        for (int q = 0; q < 8; ++q) G.lanes[q] = lg->lanes[q];
      }
      tab = t < tabs.size() ? (uint32_t)t + 1 : 0;
    }
    const bool smem_ok = lg ? (tab != 0 && (lg->nb == 32 || lg->nb == 64)) : smem_dev;
    if (kind[i] == IK_GMEM || (kind[i] == IK_SMEM && smem_ok)) {
      const TMem& m = k.mems[in.mem];
      IngJob jb{};
      jb.pad0 = (uint8_t)tab;
      jb.mask = in.mask;
      jb.base = m.base;
      jb.stride = m.stride;
      jb.list = m.list;
      jb.width = in.width;
      jb.kind = kind[i];
      job_of[i] = (uint32_t)jobs.size();
      jobs.push_back(jb);
    }
  }
  std::vector<uint32_t> res(jobs.size()), offs(jobs.size()), nmf(jobs.size());
  std::vector<TAcc> dacc;
  const auto td0 = std::chrono::steady_clock::now();
  if (!jobs.empty()) {
    IngestCtx& X = ctx();
    X.bind(device);
    hipStream_t s = X.stream;
    constexpr size_t kBatch = 1u << 16;
    const size_t nb_jobs = std::min(jobs.size(), kBatch);
    X.addrs.ensure(k.addrs.size() * sizeof(uint64_t));
    if (!k.addrs.empty())
      IHIPCHECK(hipMemcpyAsync(X.addrs.p, k.addrs.data(), k.addrs.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    X.jobs.ensure(nb_jobs * sizeof(IngJob));
    X.res.ensure(nb_jobs * 4);
    X.offs.ensure(nb_jobs * 4);
    X.nmf.ensure(nb_jobs * 4);
    X.acc.ensure(nb_jobs * kMaxAccess * sizeof(TAcc));
    X.cur.ensure(4);
    for (size_t b0 = 0; b0 < jobs.size(); b0 += kBatch) {
      const uint32_t nj = (uint32_t)std::min(kBatch, jobs.size() - b0);
      IHIPCHECK(hipMemcpyAsync(X.jobs.p, jobs.data() + b0, nj * sizeof(IngJob), hipMemcpyHostToDevice, s));
      IHIPCHECK(hipMemsetAsync(X.cur.p, 0, 4, s));
      const uint32_t groups = (nj + kWavesPerGroup - 1) / kWavesPerGroup;
      hipLaunchKernelGGL(ingest_kernel, dim3(groups), dim3(64 * kWavesPerGroup), 0, s, X.jobs.get<IngJob>(), nj,
                         X.addrs.get<uint64_t>(), prm, X.res.get<uint32_t>(), X.offs.get<uint32_t>(),
                         X.nmf.get<uint32_t>(), X.acc.get<TAcc>(), X.cur.get<uint32_t>());
      IHIPCHECK(hipGetLastError());
      IHIPCHECK(hipMemcpyAsync(res.data() + b0, X.res.p, nj * 4, hipMemcpyDeviceToHost, s));
      IHIPCHECK(hipMemcpyAsync(offs.data() + b0, X.offs.p, nj * 4, hipMemcpyDeviceToHost, s));
      IHIPCHECK(hipMemcpyAsync(nmf.data() + b0, X.nmf.p, nj * 4, hipMemcpyDeviceToHost, s));
      IHIPCHECK(hipMemcpyAsync(X.h_cur, X.cur.p, 4, hipMemcpyDeviceToHost, s));
      IHIPCHECK(hipStreamSynchronize(s));
      const uint32_t used = *X.h_cur;
      const size_t base = dacc.size();
      dacc.resize(base + used);
      if (used) {
        IHIPCHECK(hipMemcpyAsync(dacc.data() + base, X.acc.p, used * sizeof(TAcc), hipMemcpyDeviceToHost, s));
        IHIPCHECK(hipStreamSynchronize(s));
      }
      for (uint32_t q = 0; q < nj; ++q)  // batch-local offsets -> offsets into dacc
        if (jobs[b0 + q].kind == IK_GMEM && res[b0 + q] != kFallback) offs[b0 + q] += (uint32_t)base;
    }
  }
  const auto td1 = std::chrono::steady_clock::now();
  // assemble in instruction order (accesses are laid out in that order)
  std::vector<uint64_t> lane(64);
  TAcc tmp[kMaxAccess];
  IngestStats loc;
  for (size_t i = 0; i < n; ++i) {
    TInst& in = r.insts[i];
    const uint32_t jb = job_of[i];
    switch (kind[i]) {
      case IK_DONE:
        break;
      case IK_SCALAR:
        ingest_scalar(in, c, name_hash, r.accs);
        break;
      case IK_SMEM:
        if (jb != kNoMem && res[jb] != kFallback) {
          ++loc.smem_jobs;
          loc.mfma += nmf[jb];
          in.width = (uint8_t)std::min<uint32_t>(255, res[jb]);
        } else {
          ++loc.smem_host;
          ingest_lane_addresses(k, in, lane.data(), ws);
          in.width = (uint8_t)std::min<uint32_t>(
              255, smem_conflict_degree(lane.data(), in.mask, in.width ? in.width : 4, c, ws, lds_groups(c, in.opcode, ws)));
        }
        in.mem = kNoMem;
        break;
      case IK_GMEM:
        if (res[jb] != kFallback) {
          ++loc.gmem_jobs;
          loc.mfma += nmf[jb];
          ingest_finish_global(in, dacc.data() + (res[jb] ? offs[jb] : 0), res[jb], r.accs);
        } else {
          ++loc.gmem_host;
          ingest_lane_addresses(k, in, lane.data(), ws);
          const uint32_t na = coalesce_lanes(lane.data(), in.mask, in.width ? in.width : 4, ws, c, tmp);
          ingest_finish_global(in, tmp, na, r.accs);
        }
        break;
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  if (st) {
    st->smem_jobs += loc.smem_jobs;
    st->smem_host += loc.smem_host;
    st->gmem_jobs += loc.gmem_jobs;
    st->gmem_host += loc.gmem_host;
    st->mfma += loc.mfma;
    st->device_s += std::chrono::duration<double>(td1 - td0).count();
    st->total_s += std::chrono::duration<double>(t1 - t0).count();
  }
  return true;
}

}  // namespace asim

namespace asim {
int gpu_current_device() {
  int ndev = 0, d = -1;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -1;
  if (hipGetDevice(&d) != hipSuccess) return -1;
  return d;
}
}  // namespace asim
