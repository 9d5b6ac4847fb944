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
// One wave per simulated rank, one lane per xGMI link of that rank (see Wave
// below); several ranks of one process (the in-process emulation used by the
// tests and the loopback bench) are several blocks of the same launch.
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

// LDS-typed pointers: their loads wait only for LDS traffic, where a generic
// (flat) load must also drain every outstanding global store first -- in the
// packing loop, one HBM round trip per packet
#define LDS_AS __attribute__((address_space(3)))
// and HBM-typed store targets: a generic store may alias LDS, so every later
// LDS load would have to wait for it to land
#define GLB_AS __attribute__((address_space(1)))

__device__ __forceinline__ void store_pkt_g(GLB_AS int64_t* w, const LinkPkt& p) {
  int64_t v[4];
  __builtin_memcpy(v, &p, sizeof(v));
  w[0] = v[0];
  w[1] = v[1];
  w[2] = v[2];
  w[3] = v[3];
}

struct Rank {
  DlsState* s;
  LsReady* heap;  // per-link heaps at s->lheap_off[l] (HBM)
  LinkPkt* pk;    // per-link emitted packets, same offsets (HBM)
  int64_t* extra;
  int64_t* extra_words_g;
  // per-destination counters, overflow sizes and links, in LDS
  LDS_AS int64_t* cnt;
  LDS_AS int64_t* fill;
  LDS_AS int64_t* extra_words;
  LDS_AS int64_t* base;  // start of each destination's overflow words
  LDS_AS int32_t* dlink;
};

__device__ Rank rank_view(char* base, const DlsLayout& L) {
  Rank r;
  r.s = reinterpret_cast<DlsState*>(base);
  r.heap = reinterpret_cast<LsReady*>(base + L.off_heap);
  r.pk = reinterpret_cast<LinkPkt*>(base + L.off_pk);
  r.extra = reinterpret_cast<int64_t*>(base + L.off_extra);
  r.extra_words_g = reinterpret_cast<int64_t*>(base + L.off_ew);
  r.cnt = r.fill = r.extra_words = r.base = nullptr;
  r.dlink = nullptr;
  return r;
}

__device__ __forceinline__ int64_t wave_min(int64_t v) {
  for (int m = 32; m >= 1; m >>= 1) v = min(v, (int64_t)__shfl_xor((long)v, m));
  return v;
}
__device__ __forceinline__ int64_t wave_max(int64_t v) {
  for (int m = 32; m >= 1; m >>= 1) v = max(v, (int64_t)__shfl_xor((long)v, m));
  return v;
}
__device__ __forceinline__ int64_t wave_sum(int64_t v) {
  for (int m = 32; m >= 1; m >>= 1) v += (int64_t)__shfl_xor((long)v, m);
  return v;
}

__device__ __forceinline__ int64_t clamp_i64(uint64_t t) { return t > (uint64_t)kDlsI64Max ? kDlsI64Max : (int64_t)t; }

// The wave's registers hold the rank's scalar state for one launch; lane l
// owns link l: its pending sends (a heap), its clock, and the destinations it
// carries (ls_link_of(d) == l).  On one link the host LinkSim's emit order
// reduces to "pop while the head is due and the link is free before t_end"
// (a blocked link blocks every later send on it, and links never interact), so
// the links run in parallel and no send is popped only to be deferred.
struct Wave {
  int lane;
  bool own;      // lane < links
  int32_t hn;    // this link's heap size
  uint64_t lf;   // this link's clock
  LsReady* h;    // this link's heap
  LinkPkt* out;  // this link's packets of the epoch
  bool out_lds;  // ... staged in LDS
  // uniform copies
  uint64_t recv_left, send_left, sent, finish;
  int64_t t, t_end, ann_next, ann_busy;
  uint64_t epochs, packets;
  int32_t status;
};

// false on every lane if the push onto link l would overflow its heap
__device__ bool cap_ok(const DlsState& s, const Wave& w, int l) {
  const bool bad = w.own && w.lane == l && w.hn >= s.lheap_cap[w.lane];
  return !__any(bad);
}

// unpack_epoch: deliver the received slots (sources in rank order, each in
// emission order, the overflow words after a source's slot packets)
__device__ bool unpack(const Rank& R, Wave& w, const int64_t* recv, int64_t src_stride, const int64_t* spill,
                       int64_t spill_words, bool with_spill) {
  const DlsState& s = *R.s;
  const LsGeom& g = s.g;
  const int W = g.world, K = s.k, H = s.hdr;
  int64_t maxc = 0;
  for (int r = 0; r < W; ++r) maxc = max(maxc, recv[r * src_stride + 1]);
  if (maxc > K && !with_spill) {
    // some rank sent more than K packets to one destination: every rank sees
    // it in the headers and stops here for the overflow exchange
    w.status = DLS_SPILL;
    return false;
  }
  int64_t any_busy = 0, nxt = kDlsI64Max, off = 0;
  for (int r = 0; r < W; ++r) {
    const int64_t* hd = recv + r * src_stride;
    const int64_t n = hd[0];
    const int64_t in_slot = min<int64_t>(n, K);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t* wp;
      if (i < in_slot) {
        wp = hd + H + 4 * i;
      } else {
        if (!with_spill || off + 4 > spill_words) {
          w.status = DLS_ERR_SPILL;
          return false;
        }
        wp = spill + off;
        off += 4;
      }
      const LinkPkt pk = load_pkt(wp);
      if (pk.dst != g.rank) {
        w.status = DLS_ERR_DST;
        return false;
      }
      if (ls_recv_peer(g, pk.chan, pk.step) != pk.src) {
        w.status = DLS_ERR_SRC;
        return false;
      }
      // LinkSim::receive
      const uint64_t done = pk.arrive_ps + ls_local_ps(g, pk.bytes, pk.step);
      if (done > w.finish) w.finish = done;
      --w.recv_left;
      const int k1 = pk.step + 1;
      const int nd = ls_forwards(g) ? ls_send_peer(g, pk.chan, k1) : -1;
      if (nd >= 0) {
        const int l = R.dlink[nd];
        if (!cap_ok(s, w, l)) {
          w.status = DLS_ERR_CAP;
          return false;
        }
        if (w.own && l == w.lane) heap_push(w.h, w.hn, LsReady{done, pk.chan, k1, pk.slice, 0});
      }
    }
    any_busy = max(any_busy, hd[3]);
    nxt = min(nxt, min(hd[2], hd[4]));
  }
  ++w.epochs;
  if (!any_busy) {  // every rank was done before this epoch
    w.status = DLS_DONE;
    return false;
  }
  w.ann_next = wave_min(w.own && w.hn > 0 ? clamp_i64(w.h[0].t) : kDlsI64Max);
  w.ann_busy = (w.recv_left == 0 && w.send_left == 0) ? 0 : 1;
  if (nxt >= kDlsI64Max) {  // no pending send anywhere and nothing on the wire, yet a rank is not done
    w.status = DLS_ERR_DEADLOCK;
    return false;
  }
  w.t = max(w.t_end, nxt);
  return true;
}

__device__ __forceinline__ LinkPkt read_pkt(const LDS_AS LinkPkt* p) {
  const LDS_AS int64_t* w = (const LDS_AS int64_t*)p;
  const int64_t v[4] = {w[0], w[1], w[2], w[3]};
  LinkPkt q;
  __builtin_memcpy(&q, v, sizeof(q));
  return q;
}
__device__ __forceinline__ LinkPkt read_pkt(const LinkPkt* p) { return *p; }

// the lane's packets into its destinations' slots, emission order per
// destination (past K: overflow words, destination order)
template <class PktPtr>
__device__ void pack_store(const Rank& R, PktPtr out, int32_t npk, int64_t* send, int64_t slot) {
  const DlsState& s = *R.s;
  const int K = s.k, H = s.hdr;
  GLB_AS int64_t* gsend = (GLB_AS int64_t*)send;
  GLB_AS int64_t* gextra = (GLB_AS int64_t*)R.extra;
  for (int i = 0; i < npk; ++i) {
    const LinkPkt p = read_pkt(out + i);
    const int d = p.dst;
    const int64_t f = R.fill[d]++;
    if (f < K)
      store_pkt_g(gsend + d * slot + H + 4 * f, p);
    else
      store_pkt_g(gextra + R.base[d] + 4 * (f - K), p);
  }
}

// LinkSim::emit + pack_epoch for the epoch [t, t + E)
__device__ void pack(const Rank& R, Wave& w, int64_t* send, uint64_t* tp) {
  const DlsState& s = *R.s;
  const LsGeom& g = s.g;
  const int W = g.world, K = s.k, H = s.hdr;
  const int64_t slot = H + 4 * K;
  const uint64_t t_end = (uint64_t)w.t + g.epoch_ps;
  w.t_end = (int64_t)t_end;
  int32_t npk = 0;
  uint64_t fin = 0;
  int64_t min_arr = kDlsI64Max;
  if (w.own) {
    while (w.hn > 0 && w.h[0].t < t_end && w.lf < t_end) {
      const LsReady r = heap_pop(w.h, w.hn);
      const int dst = ls_send_peer(g, r.chan, r.step);
      const uint64_t st = max(r.t, w.lf);
      const uint32_t b = ls_slice_len(g, r.slice);
      const uint64_t ser = ls_ser_ps(g, b);
      w.lf = st + ser;
      LinkPkt p;
      p.src = g.rank;
      p.dst = dst;
      p.chan = r.chan;
      p.step = r.step;
      p.slice = r.slice;
      p.bytes = b;
      p.arrive_ps = st + ser + g.lat_ps;
      w.out[npk++] = p;
      fin = max(fin, st + ser);
      min_arr = min(min_arr, clamp_i64(p.arrive_ps));
    }
    for (int d = 0; d < W; ++d)
      if (R.dlink[d] == w.lane) R.cnt[d] = R.fill[d] = 0;
    for (int i = 0; i < npk; ++i) ++R.cnt[w.out[i].dst];
  }
  tp[0] = clock64();
  const int64_t tot = wave_sum(npk);
  w.send_left -= (uint64_t)tot;
  w.sent += (uint64_t)tot;
  w.finish = max(w.finish, (uint64_t)wave_max((int64_t)fin));
  min_arr = wave_min(min_arr);
  int64_t mx_l = 0;
  if (w.own)
    for (int d = 0; d < W; ++d)
      if (R.dlink[d] == w.lane) {
        mx_l = max(mx_l, R.cnt[d]);
        R.extra_words[d] = R.cnt[d] > K ? 4 * (R.cnt[d] - K) : 0;
      }
  const int64_t mx = wave_max(mx_l);
  __syncthreads();  // every link's overflow sizes are out
  int64_t ex = 0;
  for (int d = 0; d < W; ++d) ex += R.extra_words[d];
  if (w.own) {
    for (int d = 0; d < W; ++d) {
      if (R.dlink[d] != w.lane) continue;
      int64_t b0 = 0;  // destination order
      for (int e = 0; e < d; ++e) b0 += R.extra_words[e];
      R.base[d] = b0;
    }
  }
  // every slot's header and unused packet words, one word per lane: a lane
  // writing them alone issued ~40 one-lane stores per destination and stalled
  // on the outstanding-store limit
  {
    GLB_AS int64_t* gsend = (GLB_AS int64_t*)send;
    const int sl = (int)slot;  // 32-bit index math: a 64-bit division is a long instruction sequence
    for (int i = w.lane; i < W * sl; i += 64) {
      const int d = i / sl;
      const int j = i - d * sl;
      int64_t v = 0;
      if (j == 0) v = R.cnt[d];
      else if (j == 1) v = mx;
      else if (j == 2) v = w.ann_next;
      else if (j == 3) v = w.ann_busy;
      else if (j == 4) v = min_arr;
      else if (j >= H && (j - H) / 4 < min<int64_t>(R.cnt[d], K)) continue;  // a packet goes there
      gsend[i] = v;
    }
  }
  tp[1] = clock64();
  if (w.own) {
    if (w.out_lds)
      pack_store(R, (const LDS_AS LinkPkt*)w.out, npk, send, slot);
    else
      pack_store(R, (const LinkPkt*)w.out, npk, send, slot);
  }
  tp[2] = clock64();
  w.packets += (uint64_t)tot;
  R.s->extra_total = ex;  // uniform value
}

// LDS per epoch block: the rank header, its received slots, per-destination
// counters and -- when they fit -- the links' heaps and packet buffers, so the
// dependent chains of the event work hit LDS instead of HBM (the state was
// written by the previous launch, often on another XCD's L2)
constexpr int kLdsBytes = 60 * 1024;  // + the static reg_off: under the 64 KB default limit
static_assert(sizeof(DlsState) % 8 == 0 && sizeof(LsReady) % 8 == 0, "copied in 8-byte words");

__device__ __forceinline__ size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// cooperative copies of n 8-byte words between HBM and LDS (typed, so the
// loads of one pass are not serialised behind the stores of the last)
__device__ __forceinline__ void copy_in(LDS_AS int64_t* dst, const GLB_AS int64_t* src, int64_t n, int lane) {
  for (int64_t i = lane; i < n; i += 64) dst[i] = src[i];
}
__device__ __forceinline__ void copy_out(GLB_AS int64_t* dst, const LDS_AS int64_t* src, int64_t n, int lane) {
  for (int64_t i = lane; i < n; i += 64) dst[i] = src[i];
}

__global__ void __launch_bounds__(64) dls_epoch_kernel(char* states, DlsLayout L, const int64_t* recv,
                                                       int64_t recv_src_stride, int64_t recv_rank_stride,
                                                       int64_t* send, int64_t send_rank_stride, const int64_t* spill,
                                                       const int64_t* spill_off, const int64_t* t0, int mode) {
  extern __shared__ __align__(16) char lds[];
  __shared__ int64_t reg_off[kLsMaxLinks + 1];
  const int b = blockIdx.x, lane = threadIdx.x;
  const uint64_t c0 = clock64();
  const Rank G = rank_view(states + (size_t)b * L.bytes, L);
  const bool with_spill = mode == DLS_MODE_SPILL;
  {
    const int32_t st = G.s->status;
    if (mode == DLS_MODE_FIRST ? st != DLS_RUN : with_spill ? st != DLS_SPILL : st != DLS_RUN) return;
  }
  // header and received slots to LDS
  DlsState& s = *reinterpret_cast<DlsState*>(lds);
  copy_in((LDS_AS int64_t*)lds, (const GLB_AS int64_t*)G.s, sizeof(DlsState) / 8, lane);
  __syncthreads();
  const int W = s.g.world;
  const int64_t slot = s.hdr + 4 * s.k;
  size_t o = al16(sizeof(DlsState));
  int64_t* lrecv = reinterpret_cast<int64_t*>(lds + o);
  o = al16(o + (size_t)W * slot * 8);
  if (mode != DLS_MODE_FIRST) {
    const int64_t* rv = recv + b * recv_rank_stride;
    const GLB_AS int64_t* grv = (const GLB_AS int64_t*)rv;
    LDS_AS int64_t* lrv = (LDS_AS int64_t*)lrecv;
    const int sl = (int)slot;
    for (int i = lane; i < W * sl; i += 64) {
      const int r = i / sl;
      lrv[i] = grv[r * recv_src_stride + (i - r * sl)];
    }
  }
  Rank R = G;
  R.s = &s;
  R.cnt = (LDS_AS int64_t*)(lds + o);
  R.fill = R.cnt + W;
  R.extra_words = R.fill + W;
  R.base = R.extra_words + W;
  o = al16(o + (size_t)4 * W * 8);
  R.dlink = (LDS_AS int32_t*)(lds + o);
  o = al16(o + (size_t)W * 4);
  for (int d = lane; d < W; d += 64) R.dlink[d] = ls_link_of(s.g, d);
  __syncthreads();
  // links' heaps (+ this epoch's pushes) and packet buffers in LDS when they fit
  const int nl = s.g.nlinks;
  int64_t P = 0;  // pushes this epoch: at most one per received packet
  if (mode != DLS_MODE_FIRST)
    for (int r = 0; r < W; ++r) P += lrecv[r * slot];
  if (lane == 0) {
    int64_t acc = 0;
    for (int l = 0; l < nl; ++l) {
      reg_off[l] = acc;
      acc += min<int64_t>(s.lheap_n[l] + P, s.lheap_cap[l]);
    }
    reg_off[nl] = acc;
  }
  __syncthreads();
  const int64_t items = reg_off[nl];
  const bool in_lds = o + (size_t)items * (sizeof(LsReady) + sizeof(LinkPkt)) <= (size_t)kLdsBytes;
  LsReady* lheap = reinterpret_cast<LsReady*>(lds + o);
  LinkPkt* lpk = reinterpret_cast<LinkPkt*>(lds + o + (size_t)items * sizeof(LsReady));
  if (in_lds) {
    // flattened over links so the loads are independent
    for (int l = 0; l < nl; ++l)
      copy_in((LDS_AS int64_t*)(lheap + reg_off[l]), (const GLB_AS int64_t*)(G.heap + s.lheap_off[l]),
              (int64_t)s.lheap_n[l] * (sizeof(LsReady) / 8), lane);
  }
  Wave w;
  w.lane = lane;
  w.own = lane < nl;
  w.hn = w.own ? s.lheap_n[lane] : 0;
  w.lf = w.own ? s.link_free[lane] : 0;
  w.out_lds = in_lds;
  if (in_lds) {
    w.h = lheap + (w.own ? reg_off[lane] : 0);
    w.out = lpk + (w.own ? reg_off[lane] : 0);
  } else {
    w.h = G.heap + (w.own ? s.lheap_off[lane] : 0);
    w.out = G.pk + (w.own ? s.lheap_off[lane] : 0);
  }
  w.recv_left = s.recv_left;
  w.send_left = s.send_left;
  w.sent = s.sent;
  w.finish = s.finish_ps;
  w.t = s.t;
  w.t_end = s.t_end;
  w.ann_next = s.ann_next;
  w.ann_busy = s.ann_busy;
  w.epochs = s.epochs;
  w.packets = s.packets;
  w.status = DLS_RUN;
  __syncthreads();
  int64_t* my_send = send + b * send_rank_stride;
  bool go = true;
  const uint64_t c1 = clock64();
  if (mode == DLS_MODE_FIRST)
    w.t = *t0;
  else
    go = unpack(R, w, lrecv, slot, with_spill ? spill + spill_off[b] : nullptr,
                with_spill ? spill_off[b + 1] - spill_off[b] : 0, with_spill);
  const uint64_t c2 = clock64();
  uint64_t tp[3] = {0, 0, 0};
  if (go) pack(R, w, my_send, tp);
  __syncthreads();
  const uint64_t c3 = clock64();
  // state back to HBM
  if (w.own) {
    s.lheap_n[lane] = w.hn;
    s.link_free[lane] = w.lf;
  }
  if (lane == 0) {
    s.recv_left = w.recv_left;
    s.send_left = w.send_left;
    s.sent = w.sent;
    s.finish_ps = w.finish;
    s.t = w.t;
    s.t_end = w.t_end;
    s.ann_next = w.ann_next;
    s.ann_busy = w.ann_busy;
    s.epochs = w.epochs;
    s.packets = w.packets;
    s.status = w.status;
  }
  __syncthreads();
  if (in_lds)
    for (int l = 0; l < nl; ++l)
      copy_out((GLB_AS int64_t*)(G.heap + s.lheap_off[l]), (const LDS_AS int64_t*)(lheap + reg_off[l]),
               (int64_t)s.lheap_n[l] * (sizeof(LsReady) / 8), lane);
  if (go)  // pack ran: this epoch's overflow sizes (an epoch stopped for the overflow exchange keeps the last ones)
    for (int i = lane; i < W; i += 64) G.extra_words_g[i] = R.extra_words[i];
  if (lane == 0) {
    s.prof[0] += c1 - c0;
    s.prof[1] += c2 - c1;
    s.prof[2] += c3 - c2;
    s.prof[3] += clock64() - c3;  // up to here; the header copy itself is not counted
    if (go) {
      s.prof[4] += tp[0] - c2;
      s.prof[5] += tp[1] - tp[0];
      s.prof[6] += tp[2] - tp[1];
    }
  }
  __syncthreads();
  copy_out((GLB_AS int64_t*)G.s, (const LDS_AS int64_t*)lds, sizeof(DlsState) / 8, lane);
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

// sends of the rank's whole schedule per link: a bound on that link's pending sends
static void link_sends(const LsGeom& g, uint64_t* per_link) {
  for (int l = 0; l < g.nlinks; ++l) per_link[l] = 0;
  for (int ch = 0; ch < g.nch; ++ch)
    for (int k = 0; k < g.nsteps; ++k) {
      const int d = ls_send_peer(g, ch, k);
      if (d >= 0) per_link[ls_link_of(g, d)] += g.nslices;
    }
}

int64_t dls_capacity(const LinkSim::Export& e) {
  if (e.g.nlinks > kLsMaxLinks) throw std::invalid_argument("linksim_dev: more than 64 links per GPU");
  uint64_t pl[kLsMaxLinks];
  link_sends(e.g, pl);
  int64_t c = 0;
  for (int l = 0; l < e.g.nlinks; ++l) c += (int64_t)pl[l] + 1;
  return c;
}

void dls_image(const LinkSim::Export& e, const DlsLayout& L, int k, int hdr, char* img) {
  if (e.g.nlinks > kLsMaxLinks) throw std::invalid_argument("linksim_dev: more than 64 links per GPU");
  // the header, the received slots and the per-destination counters stay in LDS
  if (((sizeof(DlsState) + 15) & ~(size_t)15) + (size_t)e.g.world * ((hdr + 4 * k + 4) * 8 + 4) + 48 > (size_t)kLdsBytes)
    throw std::invalid_argument("linksim_dev: too many ranks for the device epoch loop");
  std::memset(img, 0, L.bytes);
  DlsState& s = *reinterpret_cast<DlsState*>(img);
  s.g = e.g;
  for (size_t i = 0; i < e.link_free.size(); ++i) s.link_free[i] = e.link_free[i];
  s.recv_left = e.recv_left;
  s.send_left = e.send_left;
  s.sent = e.sent;
  s.finish_ps = e.finish_ps;
  s.k = k;
  s.hdr = hdr;
  s.status = DLS_RUN;
  uint64_t pl[kLsMaxLinks];
  link_sends(e.g, pl);
  int64_t off = 0;
  for (int l = 0; l < e.g.nlinks; ++l) {
    s.lheap_off[l] = off;
    s.lheap_cap[l] = (int32_t)(pl[l] + 1);
    off += (int64_t)pl[l] + 1;
  }
  if (off > L.cap) throw std::invalid_argument("linksim_dev: state larger than its capacity");
  // pending sends to their links' heaps; ascending order is a valid min-heap
  LsReady* heap = reinterpret_cast<LsReady*>(img + L.off_heap);
  for (const LsReady& r : e.ready) {
    const int l = ls_link_of(e.g, ls_send_peer(e.g, r.chan, r.step));
    if (s.lheap_n[l] >= s.lheap_cap[l]) throw std::invalid_argument("linksim_dev: link heap over capacity");
    heap[s.lheap_off[l] + s.lheap_n[l]++] = r;
  }
  // announced state of the first exchange: as of the start
  s.ann_next = e.ready.empty() ? kDlsI64Max : (e.ready[0].t > (uint64_t)kDlsI64Max ? kDlsI64Max : (int64_t)e.ready[0].t);
  s.ann_busy = (e.recv_left == 0 && e.send_left == 0) ? 0 : 1;
}

void dls_launch_epoch(char* states, const DlsLayout& L, int nranks, const int64_t* recv, int64_t recv_src_stride,
                      int64_t recv_rank_stride, int64_t* send, int64_t send_rank_stride, const int64_t* spill,
                      const int64_t* spill_off, const int64_t* t0, int mode, void* stream) {
  hipLaunchKernelGGL(dls_epoch_kernel, dim3(nranks), dim3(64), kLdsBytes, (hipStream_t)stream, states, L, recv,
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
