// Device-resident epoch loop of the packet collective (verdict r5 item 9).
//
// The host epoch loop (exchange.cc exchange_run, parallel/collectives.py)
// bounced every epoch through the host: LinkSim emitted packets into pinned
// memory, an async copy took them to the device, RCCL exchanged them, a copy
// brought the received slots back and a stream sync handed them to LinkSim --
// one host round trip per 1 us of simulated link time.  Here each rank's
// LinkSim state (schedule geometry, pending-send heap, link clocks, counters)
// lives in HBM and one small kernel per epoch consumes the previous
// all-to-all's slots and packs the next epoch's packets in place, so an epoch
// is (kernel, all-to-all) on one HIP stream with no host involvement; the host
// only reads a status word every few epochs.  The packet rules are the host
// LinkSim's own (linksim_core.h, single source), the slot layout is
// pack_epoch / unpack_epoch's, so the results are bit-identical.
//
// One block per simulated rank, lane 0 of it runs the rank's (inherently
// serial, tens of packets per epoch) event work; several ranks of one process
// (the in-process emulation used by the tests and the loopback bench) are
// several blocks of the same launch.
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "parallel/linksim_dev.h"

namespace asim {

namespace {

__device__ __forceinline__ LinkPkt load_pkt(const int64_t* w) {
  LinkPkt p;
  __builtin_memcpy(&p, w, sizeof(p));
  return p;
}

__device__ __forceinline__ void store_pkt(int64_t* w, const LinkPkt& p) { __builtin_memcpy(w, &p, sizeof(p)); }

__device__ void heap_push(LsReady* h, int32_t& n, const LsReady& v) {
  int i = n++;
  while (i > 0) {
    const int p = (i - 1) >> 1;
    if (!ls_before(v, h[p])) break;
    h[i] = h[p];
    i = p;
  }
  h[i] = v;
}

__device__ LsReady heap_pop(LsReady* h, int32_t& n) {
  const LsReady top = h[0];
  const LsReady last = h[--n];
  int i = 0;
  for (;;) {
    const int l = 2 * i + 1;
    if (l >= n) break;
    const int r = l + 1;
    const int m = (r < n && ls_before(h[r], h[l])) ? r : l;
    if (!ls_before(h[m], last)) break;
    h[i] = h[m];
    i = m;
  }
  if (n > 0) h[i] = last;
  return top;
}

struct Rank {
  DlsState* s;
  LsReady* heap;
  LsReady* def;
  LinkPkt* pk;
  int64_t* extra;
  int64_t* extra_words;
  int64_t* cnt;
  int64_t* fill;
};

__device__ Rank rank_view(char* base, const DlsLayout& L) {
  Rank r;
  r.s = reinterpret_cast<DlsState*>(base);
  r.heap = reinterpret_cast<LsReady*>(base + L.off_heap);
  r.def = reinterpret_cast<LsReady*>(base + L.off_def);
  r.pk = reinterpret_cast<LinkPkt*>(base + L.off_pk);
  r.extra = reinterpret_cast<int64_t*>(base + L.off_extra);
  r.extra_words = reinterpret_cast<int64_t*>(base + L.off_ew);
  r.cnt = reinterpret_cast<int64_t*>(base + L.off_cnt);
  r.fill = reinterpret_cast<int64_t*>(base + L.off_fill);
  return r;
}

__device__ __forceinline__ int64_t next_event(const Rank& R) {
  if (R.s->heap_n == 0) return kDlsI64Max;
  const uint64_t t = R.heap[0].t;
  return t > (uint64_t)kDlsI64Max ? kDlsI64Max : (int64_t)t;
}

// LinkSim::receive for one packet; false (and an error status) on a bad packet
__device__ bool receive(const Rank& R, const LinkPkt& pk) {
  DlsState& s = *R.s;
  const LsGeom& g = s.g;
  if (pk.dst != g.rank) {
    s.status = DLS_ERR_DST;
    return false;
  }
  if (ls_recv_peer(g, pk.chan, pk.step) != pk.src) {
    s.status = DLS_ERR_SRC;
    return false;
  }
  const uint64_t done = pk.arrive_ps + ls_local_ps(g, pk.bytes, pk.step);
  if (done > s.finish_ps) s.finish_ps = done;
  --s.recv_left;
  const int k1 = pk.step + 1;
  if (ls_forwards(g) && ls_send_peer(g, pk.chan, k1) >= 0) {
    if (s.heap_n >= s.cap) {
      s.status = DLS_ERR_CAP;
      return false;
    }
    heap_push(R.heap, s.heap_n, LsReady{done, pk.chan, k1, pk.slice, 0});
  }
  return true;
}

// unpack_epoch: deliver the received slots (sources in rank order, each in
// emission order, the overflow words after a source's slot packets)
__device__ bool unpack(const Rank& R, const int64_t* recv, int64_t src_stride, const int64_t* spill, int64_t spill_words,
                       bool with_spill) {
  DlsState& s = *R.s;
  const int W = s.g.world, K = s.k, H = s.hdr;
  int64_t maxc = 0;
  for (int r = 0; r < W; ++r) maxc = max(maxc, recv[r * src_stride + 1]);
  if (maxc > K && !with_spill) {
    // some rank sent more than K packets to one destination: every rank sees
    // it in the headers and stops here for the host-driven overflow exchange
    s.status = DLS_SPILL;
    return false;
  }
  int64_t any_busy = 0, nxt = kDlsI64Max, off = 0;
  for (int r = 0; r < W; ++r) {
    const int64_t* h = recv + r * src_stride;
    const int64_t n = h[0];
    const int64_t in_slot = min<int64_t>(n, K);
    for (int64_t i = 0; i < in_slot; ++i)
      if (!receive(R, load_pkt(h + H + 4 * i))) return false;
    for (int64_t i = in_slot; i < n; ++i) {
      if (!with_spill || off + 4 > spill_words) {
        s.status = DLS_ERR_SPILL;
        return false;
      }
      if (!receive(R, load_pkt(spill + off))) return false;
      off += 4;
    }
    any_busy = max(any_busy, h[3]);
    nxt = min(nxt, min(h[2], h[4]));
  }
  ++s.epochs;
  if (!any_busy) {  // every rank was done before this epoch
    s.status = DLS_DONE;
    return false;
  }
  s.ann_next = next_event(R);
  s.ann_busy = (s.recv_left == 0 && s.send_left == 0) ? 0 : 1;
  if (nxt >= kDlsI64Max) {  // no pending send anywhere and nothing on the wire, yet a rank is not done
    s.status = DLS_ERR_DEADLOCK;
    return false;
  }
  s.t = max(s.t_end, nxt);
  return true;
}

// LinkSim::emit + pack_epoch for the epoch [t, t + E)
__device__ void pack(const Rank& R, int64_t* send) {
  DlsState& s = *R.s;
  const LsGeom& g = s.g;
  const int W = g.world, K = s.k, H = s.hdr;
  const int64_t slot = H + 4 * K;
  const uint64_t t_end = (uint64_t)s.t + g.epoch_ps;
  s.t_end = (int64_t)t_end;
  int32_t npk = 0, ndef = 0;
  while (s.heap_n > 0 && R.heap[0].t < t_end) {
    const LsReady r = heap_pop(R.heap, s.heap_n);
    const int dst = ls_send_peer(g, r.chan, r.step);
    const int l = ls_link_of(g, dst);
    const uint64_t st = max(r.t, s.link_free[l]);
    if (st >= t_end) {
      R.def[ndef++] = r;
      continue;
    }
    const uint32_t b = ls_slice_len(g, r.slice);
    const uint64_t ser = ls_ser_ps(g, b);
    s.link_free[l] = st + ser;
    LinkPkt p;
    p.src = g.rank;
    p.dst = dst;
    p.chan = r.chan;
    p.step = r.step;
    p.slice = r.slice;
    p.bytes = b;
    p.arrive_ps = st + ser + g.lat_ps;
    R.pk[npk++] = p;
    --s.send_left;
    ++s.sent;
    if (st + ser > s.finish_ps) s.finish_ps = st + ser;
  }
  for (int i = 0; i < ndef; ++i) heap_push(R.heap, s.heap_n, R.def[i]);
  for (int d = 0; d < W; ++d) R.cnt[d] = R.fill[d] = 0;
  int64_t min_arr = kDlsI64Max;
  for (int i = 0; i < npk; ++i) {
    ++R.cnt[R.pk[i].dst];
    const uint64_t a = R.pk[i].arrive_ps;
    min_arr = min(min_arr, a > (uint64_t)kDlsI64Max ? kDlsI64Max : (int64_t)a);
  }
  int64_t mx = 0, ex = 0;
  for (int d = 0; d < W; ++d) {
    mx = max(mx, R.cnt[d]);
    const int64_t over = R.cnt[d] > K ? 4 * (R.cnt[d] - K) : 0;
    R.extra_words[d] = over;
    R.fill[d] = 0;
    ex += over;
  }
  for (int d = 0; d < W; ++d) {
    int64_t* h = send + d * slot;
    for (int64_t i = 0; i < slot; ++i) h[i] = 0;
    h[0] = R.cnt[d];
    h[1] = mx;
    h[2] = s.ann_next;
    h[3] = s.ann_busy;
    h[4] = min_arr;
  }
  // overflow words in destination order, emission order within each
  int64_t base = 0;
  for (int d = 0; d < W; ++d) {
    R.cnt[d] = base;  // reused: start of d's overflow words
    base += R.extra_words[d];
  }
  for (int i = 0; i < npk; ++i) {
    const int d = R.pk[i].dst;
    const int64_t f = R.fill[d]++;
    if (f < K)
      store_pkt(send + d * slot + H + 4 * f, R.pk[i]);
    else
      store_pkt(R.extra + R.cnt[d] + 4 * (f - K), R.pk[i]);
  }
  s.extra_total = ex;
  s.packets += (uint64_t)npk;
}

__global__ void __launch_bounds__(64) dls_epoch_kernel(char* states, DlsLayout L, const int64_t* recv,
                                                       int64_t recv_src_stride, int64_t recv_rank_stride,
                                                       int64_t* send, int64_t send_rank_stride, const int64_t* spill,
                                                       const int64_t* spill_off, const int64_t* t0, int mode) {
  if (threadIdx.x != 0) return;
  const int b = blockIdx.x;
  const Rank R = rank_view(states + (size_t)b * L.bytes, L);
  DlsState& s = *R.s;
  int64_t* my_send = send + b * send_rank_stride;
  if (mode == DLS_MODE_FIRST) {
    if (s.status != DLS_RUN) return;
    s.t = *t0;
    pack(R, my_send);
    return;
  }
  const bool with_spill = mode == DLS_MODE_SPILL;
  if (with_spill ? s.status != DLS_SPILL : s.status != DLS_RUN) return;
  if (with_spill) s.status = DLS_RUN;
  const int64_t* my_recv = recv + b * recv_rank_stride;
  const int64_t* sp = with_spill ? spill + spill_off[b] : nullptr;
  const int64_t spw = with_spill ? spill_off[b + 1] - spill_off[b] : 0;
  if (!unpack(R, my_recv, recv_src_stride, sp, spw, with_spill)) return;
  pack(R, my_send);
}

// the in-process emulation's all-to-all: rank d's slot from rank s is rank
// s's slot for d (send [s][d][slot] -> recv [d][s][slot])
__global__ void __launch_bounds__(256) dls_transpose_kernel(const int64_t* send, int64_t* recv, int W, int slot) {
  const int64_t n = (int64_t)W * W * slot;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = i % slot, sd = i / slot, s = sd / W, d = sd % W;
    recv[(d * W + s) * slot + w] = send[i];
  }
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("linksim_dev: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

DlsLayout dls_layout(int world, int64_t cap) {
  DlsLayout L;
  const size_t c = (size_t)(cap < 1 ? 1 : cap);
  size_t o = align_up(sizeof(DlsState));
  L.off_heap = o;
  o = align_up(o + c * sizeof(LsReady));
  L.off_def = o;
  o = align_up(o + c * sizeof(LsReady));
  L.off_pk = o;
  o = align_up(o + c * sizeof(LinkPkt));
  L.off_extra = o;
  o = align_up(o + c * 4 * sizeof(int64_t));
  L.off_ew = o;
  o = align_up(o + (size_t)world * sizeof(int64_t));
  L.off_cnt = o;
  o = align_up(o + (size_t)world * sizeof(int64_t));
  L.off_fill = o;
  o = align_up(o + (size_t)world * sizeof(int64_t));
  L.bytes = o;
  L.cap = (int64_t)c;
  return L;
}

int64_t dls_capacity(const LinkSim::Export& e) {
  // every pending send is one of the collective's remaining sends
  return (int64_t)(e.send_left > e.ready.size() ? e.send_left : e.ready.size()) + 1;
}

void dls_image(const LinkSim::Export& e, const DlsLayout& L, int k, int hdr, char* img) {
  if (e.g.nlinks > kLsMaxLinks) throw std::invalid_argument("linksim_dev: more than 64 links per GPU");
  if ((int64_t)e.ready.size() > L.cap) throw std::invalid_argument("linksim_dev: state larger than its capacity");
  std::memset(img, 0, L.bytes);
  DlsState& s = *reinterpret_cast<DlsState*>(img);
  s.g = e.g;
  for (size_t i = 0; i < e.link_free.size(); ++i) s.link_free[i] = e.link_free[i];
  s.recv_left = e.recv_left;
  s.send_left = e.send_left;
  s.sent = e.sent;
  s.finish_ps = e.finish_ps;
  s.heap_n = (int32_t)e.ready.size();
  s.cap = (int32_t)L.cap;
  s.k = k;
  s.hdr = hdr;
  s.status = DLS_RUN;
  // announced state of the first exchange: as of the start
  const uint64_t ne = e.ready.empty() ? ~0ull : e.ready[0].t;
  s.ann_next = ne > (uint64_t)kDlsI64Max ? kDlsI64Max : (int64_t)ne;
  s.ann_busy = (e.recv_left == 0 && e.send_left == 0) ? 0 : 1;
  // ascending order is a valid min-heap
  std::memcpy(img + L.off_heap, e.ready.data(), e.ready.size() * sizeof(LsReady));
}

void dls_launch_epoch(char* states, const DlsLayout& L, int nranks, const int64_t* recv, int64_t recv_src_stride,
                      int64_t recv_rank_stride, int64_t* send, int64_t send_rank_stride, const int64_t* spill,
                      const int64_t* spill_off, const int64_t* t0, int mode, void* stream) {
  hipLaunchKernelGGL(dls_epoch_kernel, dim3(nranks), dim3(64), 0, (hipStream_t)stream, states, L, recv,
                     recv_src_stride, recv_rank_stride, send, send_rank_stride, spill, spill_off, t0, mode);
  check(hipGetLastError(), "epoch kernel launch");
}

void dls_launch_transpose(const int64_t* send, int64_t* recv, int world, int slot, void* stream) {
  const int64_t n = (int64_t)world * world * slot;
  const int blocks = (int)((n + 255) / 256 < 64 ? (n + 255) / 256 : 64);
  hipLaunchKernelGGL(dls_transpose_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, send,
                     recv, world, slot);
  check(hipGetLastError(), "transpose kernel launch");
}

const char* dls_status_name(int32_t st) {
  switch (st) {
    case DLS_RUN: return "running";
    case DLS_DONE: return "done";
    case DLS_SPILL: return "overflow exchange pending";
    case DLS_ERR_DST: return "packet delivered to the wrong rank";
    case DLS_ERR_SRC: return "unexpected packet source";
    case DLS_ERR_SPILL: return "overflow payload shorter than announced";
    case DLS_ERR_CAP: return "pending-send heap full";
    case DLS_ERR_DEADLOCK: return "packet collective deadlocked (no rank has pending work)";
  }
  return "unknown status";
}

}  // namespace asim
