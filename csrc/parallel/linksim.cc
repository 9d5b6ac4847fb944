#include "linksim.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstring>
#include <numeric>
#include <stdexcept>

namespace asim {

static constexpr uint64_t kNever = std::numeric_limits<uint64_t>::max();

CollKind coll_kind(const std::string& n) {
  if (n == "AllReduce") return CK_ALLREDUCE;
  if (n == "AllGather") return CK_ALLGATHER;
  if (n == "ReduceScatter") return CK_REDUCESCATTER;
  if (n == "Broadcast" || n == "Bcast") return CK_BROADCAST;
  if (n == "Reduce") return CK_REDUCE;
  if (n == "AllToAll" || n == "AlltoAll") return CK_ALLTOALL;
  if (n == "SendRecv" || n == "Send" || n == "Recv") return CK_SENDRECV;
  throw std::invalid_argument("packet collective model: unsupported collective '" + n + "'");
}

LinkSim::LinkSim(const LinkParams& p, const CollSpec& c, int rank, int world, uint64_t start_ps)
    : p_(p), finish_ps_(start_ps) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("LinkSim: bad rank/world");
  if (p.link_gbps <= 0 || p.reduce_gbps <= 0) throw std::invalid_argument("LinkSim: bandwidths must be > 0");
  const int N = world;
  g_.kind = c.kind;
  g_.root = ls_mod(c.root < 0 ? 0 : c.root, N);
  g_.rank = rank;
  g_.world = world;
  // ring strides coprime with N give disjoint rings over distinct links
  int nst = 0;
  if (N > 1) {
    const bool ring = c.kind != CK_ALLTOALL && c.kind != CK_SENDRECV;
    const uint32_t cap = ring ? std::max<uint32_t>(1, std::min(p.links, p.max_channels)) : 1;
    for (int s = 1; s < N && (uint32_t)nst < cap; ++s)
      if (std::gcd(s, N) == 1) {
        if (nst == kLsMaxStride) throw std::invalid_argument("LinkSim: more than 64 ring channels");
        g_.stride[nst++] = s;
      }
  }
  if (nst == 0) g_.stride[nst++] = 1;
  g_.nch = nst;
  uint64_t chunk = 0;
  switch (c.kind) {
    case CK_ALLREDUCE: g_.nsteps = 2 * (N - 1); chunk = c.bytes / ((uint64_t)nst * N); break;
    case CK_ALLGATHER:
    case CK_REDUCESCATTER: g_.nsteps = N - 1; chunk = c.bytes / ((uint64_t)nst * N); break;
    case CK_BROADCAST:
    case CK_REDUCE: g_.nsteps = N - 1; chunk = c.bytes / nst; break;
    case CK_ALLTOALL: g_.nsteps = N - 1; chunk = c.bytes / N; break;
    case CK_SENDRECV: g_.nsteps = N > 1 ? 1 : 0; chunk = c.bytes; break;
  }
  if (N == 1) g_.nsteps = 0;
  g_.chunk = std::max<uint64_t>(chunk, 1);
  g_.slice_bytes = std::max<uint32_t>(p.slice_bytes, 64);
  g_.nslices = (uint32_t)((g_.chunk + g_.slice_bytes - 1) / g_.slice_bytes);
  g_.ps_per_byte_link = 1000.0 / p.link_gbps;  // GB/s == bytes/ns
  g_.ps_per_byte_mem = 1000.0 / p.reduce_gbps;
  g_.lat_ps = (uint64_t)std::llround(std::max(0.0, p.latency_ns) * 1000.0);
  g_.epoch_ps = std::max<uint64_t>(g_.lat_ps, 1000);
  if (g_.lat_ps < g_.epoch_ps) g_.lat_ps = g_.epoch_ps;  // lookahead requires latency >= epoch
  g_.nlinks = (int32_t)std::max<uint32_t>(1, p.links);
  link_free_.assign((size_t)g_.nlinks, start_ps);
  for (int ch = 0; ch < g_.nch; ++ch)
    for (int k = 0; k < g_.nsteps; ++k) {
      const bool snd = send_peer(ch, k) >= 0, rcv = recv_peer(ch, k) >= 0;
      if (snd) send_left_ += g_.nslices;
      if (rcv) recv_left_ += g_.nslices;
      const bool dep = k > 0 && recv_peer(ch, k - 1) >= 0 && ls_forwards(g_);
      if (snd && !dep)
        for (uint32_t s = 0; s < g_.nslices; ++s) push_send(start_ps, ch, k, (int)s);
    }
}

int LinkSim::send_peer(int ch, int k) const { return ls_send_peer(g_, ch, k); }
int LinkSim::recv_peer(int ch, int k) const { return ls_recv_peer(g_, ch, k); }
bool LinkSim::recv_reduces(int k) const { return ls_recv_reduces(g_, k); }

void LinkSim::push_send(uint64_t t, int c, int k, int s) { ready_.push(LsReady{t, c, k, s, 0}); }

void LinkSim::emit(uint64_t t_end, std::vector<LinkPkt>& out) {
  std::vector<LsReady> deferred;
  while (!ready_.empty() && ready_.top().t < t_end) {
    LsReady r = ready_.top();
    ready_.pop();
    const int dst = send_peer(r.chan, r.step);
    const int l = ls_link_of(g_, dst);
    const uint64_t st = std::max(r.t, link_free_[l]);
    if (st >= t_end) {
      deferred.push_back(r);
      continue;
    }
    const uint32_t b = ls_slice_len(g_, r.slice);
    const uint64_t ser = ls_ser_ps(g_, b);
    link_free_[l] = st + ser;
    LinkPkt pk;
    pk.src = g_.rank;
    pk.dst = dst;
    pk.chan = r.chan;
    pk.step = r.step;
    pk.slice = r.slice;
    pk.bytes = b;
    pk.arrive_ps = st + ser + g_.lat_ps;
    out.push_back(pk);
    --send_left_;
    ++sent_;
    finish_ps_ = std::max(finish_ps_, st + ser);
  }
  for (auto& r : deferred) ready_.push(r);
}

void LinkSim::receive(const LinkPkt* p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const LinkPkt& pk = p[i];
    if (pk.dst != g_.rank) throw std::logic_error("LinkSim: packet delivered to the wrong rank");
    if (recv_peer(pk.chan, pk.step) != pk.src) throw std::logic_error("LinkSim: unexpected packet source");
    const uint64_t done = pk.arrive_ps + ls_local_ps(g_, pk.bytes, pk.step);
    finish_ps_ = std::max(finish_ps_, done);
    --recv_left_;
    const int k1 = pk.step + 1;
    if (ls_forwards(g_) && send_peer(pk.chan, k1) >= 0) push_send(done, pk.chan, k1, pk.slice);
  }
}

uint64_t LinkSim::next_event() const { return ready_.empty() ? kNever : ready_.top().t; }

LinkSim::Export LinkSim::export_state() const {
  Export e;
  e.g = g_;
  auto q = ready_;
  e.ready.reserve(q.size());
  for (; !q.empty(); q.pop()) e.ready.push_back(q.top());  // ascending order: already a valid min-heap
  e.link_free = link_free_;
  e.recv_left = recv_left_;
  e.send_left = send_left_;
  e.sent = sent_;
  e.finish_ps = finish_ps_;
  return e;
}

std::vector<uint64_t> linksim_run_local(const LinkParams& p, const CollSpec& c, const std::vector<uint64_t>& start_ps,
                                        uint64_t* epochs, uint64_t* packets) {
  const int N = (int)start_ps.size();
  std::vector<LinkSim> sims;
  sims.reserve(N);
  for (int r = 0; r < N; ++r) sims.emplace_back(p, c, r, N, start_ps[r]);
  uint64_t t = *std::min_element(start_ps.begin(), start_ps.end());
  const uint64_t E = sims[0].epoch_ps();
  uint64_t ep = 0, pk = 0;
  std::vector<std::vector<LinkPkt>> out(N);
  std::vector<LinkPkt> inbox;
  auto all_done = [&] {
    for (auto& s : sims)
      if (!s.done()) return false;
    return true;
  };
  while (!all_done()) {
    const uint64_t t_end = t + E;
    for (int r = 0; r < N; ++r) {
      out[r].clear();
      sims[r].emit(t_end, out[r]);
      pk += out[r].size();
    }
    // deliver: receiver sees sources in rank order, each in emission order
    for (int d = 0; d < N; ++d) {
      inbox.clear();
      for (int s = 0; s < N; ++s)
        for (auto& x : out[s])
          if (x.dst == d) inbox.push_back(x);
      sims[d].receive(inbox.data(), inbox.size());
    }
    uint64_t ne = kNever;
    for (auto& s : sims) ne = std::min(ne, s.next_event());
    ++ep;
    if (ne == kNever && !all_done()) throw std::logic_error("LinkSim: collective deadlocked");
    t = std::max(t_end, ne == kNever ? t_end : ne);
  }
  if (epochs) *epochs = ep;
  if (packets) *packets = pk;
  std::vector<uint64_t> fin(N);
  for (int r = 0; r < N; ++r) fin[r] = sims[r].finish_ps();
  return fin;
}

void pack_epoch(LinkSim& l, uint64_t t_end, int k, int hdr, int64_t ann_next, int64_t ann_busy, int64_t* send,
                EpochOut& out) {
  const int W = l.world();
  const size_t slot = (size_t)hdr + 4 * (size_t)k;
  std::vector<LinkPkt> pk;
  l.emit(t_end, pk);
  std::vector<int64_t> count(W, 0);
  int64_t min_arr = INT64_MAX;
  for (const LinkPkt& p : pk) {
    if (p.dst < 0 || p.dst >= W) throw std::runtime_error("pack_epoch: packet to a rank outside the group");
    ++count[p.dst];
    min_arr = std::min<int64_t>(min_arr, (int64_t)std::min<uint64_t>(p.arrive_ps, (uint64_t)INT64_MAX));
  }
  int64_t mx = 0;
  for (int64_t c : count) mx = std::max(mx, c);
  std::memset(send, 0, sizeof(int64_t) * slot * W);
  for (int d = 0; d < W; ++d) {
    int64_t* h = send + (size_t)d * slot;
    h[0] = count[d];
    h[1] = mx;
    h[2] = ann_next;
    h[3] = ann_busy;
    h[4] = min_arr;
  }
  // stable by destination: emission order within each destination
  std::vector<int64_t> fill(W, 0);
  out.extra.clear();
  out.extra_words.assign(W, 0);
  std::vector<std::vector<int64_t>> over(W);
  for (const LinkPkt& p : pk) {
    int64_t w[4];
    std::memcpy(w, &p, sizeof(w));
    if (fill[p.dst] < k) {
      std::memcpy(send + (size_t)p.dst * slot + hdr + 4 * fill[p.dst], w, sizeof(w));
    } else {
      over[p.dst].insert(over[p.dst].end(), w, w + 4);
    }
    ++fill[p.dst];
  }
  for (int d = 0; d < W; ++d) {
    out.extra_words[d] = (int64_t)over[d].size();
    out.extra.insert(out.extra.end(), over[d].begin(), over[d].end());
  }
  out.packets = pk.size();
  out.max_count = mx;
}

EpochIn unpack_epoch(LinkSim& l, const int64_t* recv, int k, int hdr, const int64_t* extra, size_t extra_words) {
  const int W = l.world();
  const size_t slot = (size_t)hdr + 4 * (size_t)k;
  std::vector<LinkPkt> in;
  size_t off = 0;
  EpochIn r;
  r.next = INT64_MAX;
  for (int s = 0; s < W; ++s) {
    const int64_t* h = recv + (size_t)s * slot;
    const int64_t n = h[0];
    const int64_t in_slot = std::min<int64_t>(n, k);
    for (int64_t i = 0; i < in_slot; ++i) {
      LinkPkt p;
      std::memcpy(&p, h + hdr + 4 * i, sizeof(p));
      in.push_back(p);
    }
    for (int64_t i = in_slot; i < n; ++i) {
      if (off + 4 > extra_words) throw std::runtime_error("unpack_epoch: overflow payload shorter than announced");
      LinkPkt p;
      std::memcpy(&p, extra + off, sizeof(p));
      off += 4;
      in.push_back(p);
    }
    r.any_busy = std::max(r.any_busy, h[3]);
    r.next = std::min(r.next, std::min(h[2], h[4]));
  }
  if (!in.empty()) l.receive(in.data(), in.size());
  return r;
}

}  // namespace asim
