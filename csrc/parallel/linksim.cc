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

static int mod(int a, int n) { return ((a % n) + n) % n; }

static int inv_mod(int s, int n) {
  for (int x = 1; x < n; ++x)
    if ((s * x) % n == 1) return x;
  return 1;
}

LinkSim::LinkSim(const LinkParams& p, const CollSpec& c, int rank, int world, uint64_t start_ps)
    : p_(p), c_(c), rank_(rank), world_(world), start_ps_(start_ps), finish_ps_(start_ps) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("LinkSim: bad rank/world");
  if (p.link_gbps <= 0 || p.reduce_gbps <= 0) throw std::invalid_argument("LinkSim: bandwidths must be > 0");
  const int N = world;
  c_.root = mod(c.root < 0 ? 0 : c.root, N);
  // ring strides coprime with N give disjoint rings over distinct links
  if (N > 1) {
    const bool ring = c.kind != CK_ALLTOALL && c.kind != CK_SENDRECV;
    const uint32_t cap = ring ? std::max<uint32_t>(1, std::min(p.links, p.max_channels)) : 1;
    for (int s = 1; s < N && stride_.size() < cap; ++s)
      if (std::gcd(s, N) == 1) stride_.push_back(s);
  }
  if (stride_.empty()) stride_.push_back(1);
  nch_ = (uint32_t)stride_.size();
  switch (c.kind) {
    case CK_ALLREDUCE: nsteps_ = 2 * (N - 1); chunk_ = c.bytes / ((uint64_t)nch_ * N); break;
    case CK_ALLGATHER:
    case CK_REDUCESCATTER: nsteps_ = N - 1; chunk_ = c.bytes / ((uint64_t)nch_ * N); break;
    case CK_BROADCAST:
    case CK_REDUCE: nsteps_ = N - 1; chunk_ = c.bytes / nch_; break;
    case CK_ALLTOALL: nsteps_ = N - 1; chunk_ = c.bytes / N; break;
    case CK_SENDRECV: nsteps_ = N > 1 ? 1 : 0; chunk_ = c.bytes; break;
  }
  if (N == 1) nsteps_ = 0;
  chunk_ = std::max<uint64_t>(chunk_, 1);
  const uint64_t sl = std::max<uint32_t>(p.slice_bytes, 64);
  nslices_ = (uint32_t)((chunk_ + sl - 1) / sl);
  ps_per_byte_link_ = 1000.0 / p.link_gbps;  // GB/s == bytes/ns
  ps_per_byte_mem_ = 1000.0 / p.reduce_gbps;
  lat_ps_ = (uint64_t)std::llround(std::max(0.0, p.latency_ns) * 1000.0);
  epoch_ps_ = std::max<uint64_t>(lat_ps_, 1000);
  if (lat_ps_ < epoch_ps_) lat_ps_ = epoch_ps_;  // lookahead requires latency >= epoch
  link_free_.assign(std::max<uint32_t>(1, p.links), start_ps);
  for (int ch = 0; ch < (int)nch_; ++ch)
    for (int k = 0; k < nsteps_; ++k) {
      const bool snd = send_peer(ch, k) >= 0, rcv = recv_peer(ch, k) >= 0;
      if (snd) send_left_ += nslices_;
      if (rcv) recv_left_ += nslices_;
      const bool dep = k > 0 && recv_peer(ch, k - 1) >= 0 && c.kind != CK_ALLTOALL && c.kind != CK_SENDRECV;
      if (snd && !dep)
        for (uint32_t s = 0; s < nslices_; ++s) push_send(start_ps, ch, k, (int)s);
    }
}

// position of this rank along a chain with stride s starting after `first`
static int chain_pos(int r, int first, int s, int N) { return mod((r - first) * inv_mod(s, N), N); }

int LinkSim::send_peer(int ch, int k) const {
  const int N = world_, r = rank_, s = stride_[ch];
  if (N <= 1 || k < 0 || k >= nsteps_) return -1;
  switch (c_.kind) {
    case CK_ALLREDUCE:
    case CK_ALLGATHER:
    case CK_REDUCESCATTER: return mod(r + s, N);
    case CK_BROADCAST: {
      const int pos = chain_pos(r, c_.root, s, N);
      return (k == pos && pos < N - 1) ? mod(r + s, N) : -1;
    }
    case CK_REDUCE: {
      const int pos = chain_pos(r, c_.root + s, s, N);  // root is last
      return (k == pos && pos < N - 1) ? mod(r + s, N) : -1;
    }
    case CK_ALLTOALL: return mod(r + k + 1, N);
    case CK_SENDRECV: return mod(r + 1, N);
  }
  return -1;
}

int LinkSim::recv_peer(int ch, int k) const {
  const int N = world_, r = rank_, s = stride_[ch];
  if (N <= 1 || k < 0 || k >= nsteps_) return -1;
  switch (c_.kind) {
    case CK_ALLREDUCE:
    case CK_ALLGATHER:
    case CK_REDUCESCATTER: return mod(r - s, N);
    case CK_BROADCAST: {
      const int pos = chain_pos(r, c_.root, s, N);
      return (pos > 0 && k == pos - 1) ? mod(r - s, N) : -1;
    }
    case CK_REDUCE: {
      const int pos = chain_pos(r, c_.root + s, s, N);
      return (pos > 0 && k == pos - 1) ? mod(r - s, N) : -1;
    }
    case CK_ALLTOALL: return mod(r - k - 1, N);
    case CK_SENDRECV: return mod(r - 1, N);
  }
  return -1;
}

bool LinkSim::recv_reduces(int k) const {
  switch (c_.kind) {
    case CK_ALLREDUCE: return k < world_ - 1;
    case CK_REDUCESCATTER:
    case CK_REDUCE: return true;
    default: return false;
  }
}

uint32_t LinkSim::slice_len(int s) const {
  const uint64_t sl = std::max<uint32_t>(p_.slice_bytes, 64);
  const uint64_t off = (uint64_t)s * sl;
  return (uint32_t)std::min<uint64_t>(sl, chunk_ - off);
}

int LinkSim::link_of(int dst) const {
  const int o = mod(dst - rank_ - 1, world_);
  return o % (int)link_free_.size();
}

void LinkSim::push_send(uint64_t t, int c, int k, int s) { ready_.push(Ready{t, c, k, s}); }

void LinkSim::emit(uint64_t t_end, std::vector<LinkPkt>& out) {
  std::vector<Ready> deferred;
  while (!ready_.empty() && ready_.top().t < t_end) {
    Ready r = ready_.top();
    ready_.pop();
    const int dst = send_peer(r.chan, r.step);
    const int l = link_of(dst);
    const uint64_t st = std::max(r.t, link_free_[l]);
    if (st >= t_end) {
      deferred.push_back(r);
      continue;
    }
    const uint32_t b = slice_len(r.slice);
    const uint64_t ser = (uint64_t)std::ceil(b * ps_per_byte_link_);
    link_free_[l] = st + ser;
    LinkPkt pk;
    pk.src = rank_;
    pk.dst = dst;
    pk.chan = r.chan;
    pk.step = r.step;
    pk.slice = r.slice;
    pk.bytes = b;
    pk.arrive_ps = st + ser + lat_ps_;
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
    if (pk.dst != rank_) throw std::logic_error("LinkSim: packet delivered to the wrong rank");
    if (recv_peer(pk.chan, pk.step) != pk.src) throw std::logic_error("LinkSim: unexpected packet source");
    const double per = recv_reduces(pk.step) ? 3.0 : 1.0;  // reduce: read mine + read recv + write
    const uint64_t done = pk.arrive_ps + (uint64_t)std::ceil(pk.bytes * per * ps_per_byte_mem_);
    finish_ps_ = std::max(finish_ps_, done);
    --recv_left_;
    const int k1 = pk.step + 1;
    if (c_.kind != CK_ALLTOALL && c_.kind != CK_SENDRECV && send_peer(pk.chan, k1) >= 0)
      push_send(done, pk.chan, k1, pk.slice);
  }
}

uint64_t LinkSim::next_event() const { return ready_.empty() ? kNever : ready_.top().t; }

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
