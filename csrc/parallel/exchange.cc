// Native epoch loop of the distributed packet collective: the lock-step
// PDES epochs of one collective (parallel/collectives.py PacketExchange.run,
// same protocol, bit-identical results) owned by C++ over a
// torch.distributed ProcessGroup -- RCCL over xGMI when the group's backend
// is "nccl" (device buffers, one fixed-size all-to-all per epoch on the
// current HIP stream), gloo on the CPU.  The Python loop paid an interpreter
// round trip, two numpy views and a torch dispatch per epoch; here the whole
// loop runs with the GIL released and the host work per epoch is the native
// pack / unpack around the all-to-all.
//
// Built as a torch C++ extension (build_native.py: _asim_dist), because it
// talks to c10d::ProcessGroup directly.  The reference has no counterpart: its
// distributed fork charges a constant -nccl_allreduce_latency per
// ncclAllReduce (gpu-simulator/main.cc:116-122).
#include <torch/extension.h>
#include <c10/core/impl/VirtualGuardImpl.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/utils/pybind.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

#include "linksim.h"
#include "linksim_dev.h"

namespace asim {
namespace {

constexpr int kSlots = 8;  // packet slots per destination in the fixed exchange (collectives.py K)
constexpr int kHdr = 8;    // header words per destination slot (collectives.py HDR)
constexpr int64_t kI64Max = std::numeric_limits<int64_t>::max();

LinkParams params_from(const py::dict& d) {
  LinkParams p;
  if (d.contains("link_gbps")) p.link_gbps = d["link_gbps"].cast<double>();
  if (d.contains("latency_ns")) p.latency_ns = d["latency_ns"].cast<double>();
  if (d.contains("links")) p.links = d["links"].cast<uint32_t>();
  if (d.contains("slice_bytes")) p.slice_bytes = d["slice_bytes"].cast<uint32_t>();
  if (d.contains("max_channels")) p.max_channels = d["max_channels"].cast<uint32_t>();
  if (d.contains("reduce_gbps")) p.reduce_gbps = d["reduce_gbps"].cast<double>();
  return p;
}

// exchange buffers: host (pinned when the group works on device tensors) and,
// for RCCL, their device twins; reused across epochs
struct Bufs {
  bool dev = false;
  at::Tensor h_send, h_recv, d_send, d_recv;
  void ensure(size_t n, int device) {
    if (h_send.defined() && (size_t)h_send.numel() == n) return;
    auto ho = at::TensorOptions().dtype(at::kLong).pinned_memory(dev);
    h_send = at::empty({(int64_t)n}, ho);
    h_recv = at::empty({(int64_t)n}, ho);
    if (dev) {
      auto dopt = at::TensorOptions().dtype(at::kLong).device(at::kCUDA, device);
      d_send = at::empty({(int64_t)n}, dopt);
      d_recv = at::empty({(int64_t)n}, dopt);
    }
  }
};

// one all-to-all of int64 words with the given split sizes.  RCCL: the
// pinned send words go up and the received words come back as asynchronous
// copies on the current stream, ordered around the collective (wait() only
// makes the stream wait for RCCL's), so the host blocks exactly once per
// exchange -- the stream sync before LinkSim reads the received slots.
void a2a(c10d::ProcessGroup& pg, Bufs& b, std::vector<int64_t>& out_splits, std::vector<int64_t>& in_splits) {
  at::Tensor src = b.dev ? b.d_send : b.h_send, dst = b.dev ? b.d_recv : b.h_recv;
  if (b.dev) b.d_send.copy_(b.h_send, /*non_blocking=*/true);
  auto w = pg.alltoall_base(dst, src, in_splits, out_splits);
  w->wait();
  if (b.dev) {
    b.h_recv.copy_(b.d_recv, /*non_blocking=*/true);
    const c10::impl::VirtualGuardImpl g(b.d_recv.device().type());
    g.synchronizeStream(g.getStream(b.d_recv.device()));
  }
}

int64_t allreduce_min(c10d::ProcessGroup& pg, int64_t v, bool dev, int device) {
  auto o = at::TensorOptions().dtype(at::kLong);
  at::Tensor t = at::full({1}, v, dev ? o.device(at::kCUDA, device) : o);
  std::vector<at::Tensor> ts{t};
  c10d::AllreduceOptions ao;
  ao.reduceOp = c10d::ReduceOp::MIN;
  pg.allreduce(ts, ao)->wait();
  return t.cpu().item<int64_t>();
}

}  // namespace

py::dict exchange_run(py::object pgo, py::dict params, const std::string& kind, int64_t nbytes, int64_t root,
                      int64_t start_ps, int64_t device) {
  auto pg = py::cast<c10::intrusive_ptr<c10d::ProcessGroup>>(pgo);
  const int W = pg->getSize(), R = pg->getRank();
  CollSpec cs;
  cs.kind = coll_kind(kind);
  cs.bytes = (uint64_t)nbytes;
  cs.root = (int32_t)root;
  LinkSim ls(params_from(params), cs, R, W, (uint64_t)start_ps);
  const bool dev = device >= 0;
  const int slot = kHdr + 4 * kSlots;
  const size_t n = (size_t)W * slot;
  uint64_t epochs = 0, packets = 0, exchanges = 0;
  double loop_s = 0;
  {
    py::gil_scoped_release nogil;
    const auto t0 = std::chrono::steady_clock::now();
    int64_t t = allreduce_min(*pg, std::min<int64_t>(start_ps, kI64Max), dev, (int)device);
    const int64_t E = (int64_t)ls.epoch_ps();
    int64_t ann_next = (int64_t)std::min<uint64_t>(ls.next_event(), (uint64_t)kI64Max);
    int64_t ann_busy = ls.done() ? 0 : 1;
    Bufs fixed, spill;
    fixed.dev = spill.dev = dev;
    fixed.ensure(n, (int)device);
    std::vector<int64_t> eq(W, slot);
    for (;;) {
      const int64_t t_end = t + E;
      EpochOut o;
      pack_epoch(ls, (uint64_t)t_end, kSlots, kHdr, ann_next, ann_busy, fixed.h_send.data_ptr<int64_t>(), o);
      a2a(*pg, fixed, eq, eq);
      ++exchanges;
      const int64_t* recv = fixed.h_recv.data_ptr<int64_t>();
      int64_t maxc = 0;
      for (int r = 0; r < W; ++r) maxc = std::max<int64_t>(maxc, recv[(size_t)r * slot + 1]);
      std::vector<int64_t> inc;
      if (maxc > kSlots) {
        // some rank sent more than kSlots packets to one destination: the rest
        std::vector<int64_t> in_w(W), out_w(o.extra_words.begin(), o.extra_words.end());
        size_t nin = 0;
        for (int r = 0; r < W; ++r) {
          in_w[r] = 4 * std::max<int64_t>(0, recv[(size_t)r * slot] - kSlots);
          nin += (size_t)in_w[r];
        }
        const size_t nout = o.extra.size();
        spill.h_send = at::empty({(int64_t)nout}, at::TensorOptions().dtype(at::kLong).pinned_memory(dev));
        spill.h_recv = at::empty({(int64_t)nin}, at::TensorOptions().dtype(at::kLong).pinned_memory(dev));
        if (nout) std::copy(o.extra.begin(), o.extra.end(), spill.h_send.data_ptr<int64_t>());
        if (dev) {
          auto dopt = at::TensorOptions().dtype(at::kLong).device(at::kCUDA, (int)device);
          spill.d_send = at::empty({(int64_t)nout}, dopt);
          spill.d_recv = at::empty({(int64_t)nin}, dopt);
        }
        a2a(*pg, spill, out_w, in_w);
        ++exchanges;
        inc.assign(spill.h_recv.data_ptr<int64_t>(), spill.h_recv.data_ptr<int64_t>() + nin);
      }
      const EpochIn in = unpack_epoch(ls, recv, kSlots, kHdr, inc.empty() ? nullptr : inc.data(), inc.size());
      packets += o.packets;
      ++epochs;
      if (!in.any_busy) break;  // every rank was done before this epoch
      ann_next = (int64_t)std::min<uint64_t>(ls.next_event(), (uint64_t)kI64Max);
      ann_busy = ls.done() ? 0 : 1;
      if (in.next >= kI64Max) throw std::runtime_error("packet collective deadlocked (no rank has pending work)");
      t = std::max<int64_t>(t_end, in.next);
    }
    loop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  py::dict d;
  d["finish_ps"] = ls.finish_ps();
  d["channels"] = ls.channels();
  d["packets_sent"] = ls.packets_sent();
  d["epochs"] = epochs;
  d["packets"] = packets;
  d["exchanges"] = exchanges;
  d["loop_s"] = loop_s;
  return d;
}

// per-epoch cost of the exchange primitive alone: `iters` fixed-shape
// all-to-alls of the epoch's W x (header + slots) words through the same
// a2a() path exchange_run uses (pinned host -> device -> collective -> host),
// after `warm` untimed ones; returns microseconds per exchange
// (shape_world > 0: the words of a shape_world-rank epoch, split evenly over
// this group's ranks -- on a 1-rank group a loopback of the 8-rank shape)
py::dict a2a_bench(py::object pgo, int64_t iters, int64_t warm, int64_t device, int64_t shape_world) {
  auto pg = py::cast<c10::intrusive_ptr<c10d::ProcessGroup>>(pgo);
  const int W = pg->getSize();
  const int slot = kHdr + 4 * kSlots;
  const int Wv = shape_world > 0 ? (int)shape_world : W;
  if (Wv % W) throw std::runtime_error("a2a_bench: shape_world must be a multiple of the group size");
  const size_t n = (size_t)Wv * slot;
  double s = 0;
  {
    py::gil_scoped_release nogil;
    Bufs b;
    b.dev = device >= 0;
    b.ensure(n, (int)device);
    std::vector<int64_t> eq(W, (int64_t)(n / W));
    for (size_t i = 0; i < n; ++i) b.h_send.data_ptr<int64_t>()[i] = (int64_t)i;
    for (int64_t i = 0; i < warm; ++i) a2a(*pg, b, eq, eq);
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t i = 0; i < iters; ++i) a2a(*pg, b, eq, eq);
    s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  py::dict d;
  d["us_per_exchange"] = s / (double)std::max<int64_t>(1, iters) * 1e6;
  d["iters"] = iters;
  d["words_per_rank"] = (int64_t)n;
  d["bytes_per_rank"] = (int64_t)(n * 8);
  d["world"] = W;
  d["shape_world"] = Wv;
  d["device"] = device >= 0;
  return d;
}

// ---------------------------------------------------------------------------
// Device-resident epoch loop (linksim_dev.hip): the ranks' LinkSim states live
// in HBM; an epoch is one kernel (deliver the last all-to-all's slots, pack the
// next epoch's packets into the device send buffer) and one all-to-all of
// device buffers, both on the current HIP stream.  The host enqueues epochs in
// growing batches (1, 2, 4, ... batch_max) and reads the status words once per
// batch; the epochs enqueued after the last one are no-ops on every rank (the
// termination and overflow conditions are global, so every rank stops at the
// same epoch and issues the same number of collectives).
namespace {

void sync_stream(int device) {
  const c10::impl::VirtualGuardImpl g(c10::DeviceType::CUDA);
  g.synchronizeStream(g.getStream(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device)));
}

struct DevStates {
  DlsLayout L;
  int n = 0, device = 0;
  at::Tensor blob, img, hdr;  // device state blocks; their pinned upload image; pinned copies of the headers

  void upload(const std::vector<LinkSim::Export>& ex, int world, int k, int hdr_words, int dev) {
    device = dev;
    n = (int)ex.size();
    int64_t cap = 1;
    for (auto& e : ex) cap = std::max(cap, dls_capacity(e));
    L = dls_layout(world, cap);
    const int64_t bytes = (int64_t)L.bytes * n;
    img = at::empty({bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
    for (int b = 0; b < n; ++b) dls_image(ex[b], L, k, hdr_words, (char*)img.data_ptr<uint8_t>() + (size_t)b * L.bytes);
    blob = at::empty({bytes}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
    blob.copy_(img, /*non_blocking=*/true);
    hdr = at::empty({(int64_t)sizeof(DlsState) * n}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  }
  char* base() { return (char*)blob.data_ptr<uint8_t>(); }
  // the rank headers to the host: one stream sync
  void poll() {
    for (int b = 0; b < n; ++b)
      hdr.narrow(0, (int64_t)sizeof(DlsState) * b, sizeof(DlsState))
          .copy_(blob.narrow(0, (int64_t)L.bytes * b, sizeof(DlsState)), /*non_blocking=*/true);
    sync_stream(device);
  }
  const DlsState& st(int b) const { return reinterpret_cast<const DlsState*>(hdr.data_ptr<uint8_t>())[b]; }
  // int64 words [off, off + 8 * words) of rank b's block, as a device tensor view
  at::Tensor words(int b, size_t off, int64_t nw) {
    return blob.narrow(0, (int64_t)(L.bytes * b + off), nw * 8).view(at::kLong);
  }
  int32_t status() const {
    int32_t s = st(0).status;
    for (int b = 1; b < n; ++b)
      if (st(b).status > DLS_SPILL) return st(b).status;  // a rank-local error wins
    return s;
  }
};

[[noreturn]] void dls_fail(int32_t st) { throw std::runtime_error(std::string("device epoch loop: ") + dls_status_name(st)); }


}  // namespace

py::dict exchange_run_device(py::object pgo, py::dict params, const std::string& kind, int64_t nbytes, int64_t root,
                             int64_t start_ps, int64_t device, int64_t batch_max) {
  auto pg = py::cast<c10::intrusive_ptr<c10d::ProcessGroup>>(pgo);
  const int W = pg->getSize(), R = pg->getRank();
  CollSpec cs;
  cs.kind = coll_kind(kind);
  cs.bytes = (uint64_t)nbytes;
  cs.root = (int32_t)root;
  const LinkSim ls(params_from(params), cs, R, W, (uint64_t)start_ps);
  const int slot = kHdr + 4 * kSlots;
  const int64_t n = (int64_t)W * slot;
  uint64_t exchanges = 0, polls = 0;
  double loop_s = 0;
  DevStates S;
  {
    py::gil_scoped_release nogil;
    const auto t0c = std::chrono::steady_clock::now();
    // a stream of our own; work the caller queued before is finished first
    sync_stream((int)device);
    const c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromPool(false, (c10::DeviceIndex)device));
    void* stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
    S.upload({ls.export_state()}, W, kSlots, kHdr, (int)device);
    auto dopt = at::TensorOptions().dtype(at::kLong).device(at::kCUDA, device);
    at::Tensor t0 = at::full({1}, start_ps, dopt);
    {
      std::vector<at::Tensor> ts{t0};
      c10d::AllreduceOptions ao;
      ao.reduceOp = c10d::ReduceOp::MIN;
      pg->allreduce(ts, ao)->wait();  // the stream waits; the host does not
    }
    at::Tensor d_send = at::empty({n}, dopt), d_recv = at::empty({n}, dopt);
    std::vector<int64_t> eq(W, slot);
    dls_launch_epoch(S.base(), S.L, 1, nullptr, 0, 0, d_send.data_ptr<int64_t>(), 0, nullptr, nullptr,
                     t0.data_ptr<int64_t>(), DLS_MODE_FIRST, stream);
    int64_t b = 1;
    uint64_t last_epochs = 0;

    for (;;) {
      auto one_epoch = [&] {
        pg->alltoall_base(d_recv, d_send, eq, eq)->wait();
        dls_launch_epoch(S.base(), S.L, 1, d_recv.data_ptr<int64_t>(), slot, 0, d_send.data_ptr<int64_t>(), 0, nullptr,
                         nullptr, nullptr, DLS_MODE_NEXT, stream);
      };
      for (int64_t i = 0; i < b; ++i) one_epoch();
      exchanges += (uint64_t)b;
      S.poll();
      ++polls;
      const int32_t st = S.status();
      if (st == DLS_DONE) break;
      if (st == DLS_SPILL) {
        // some rank sent more than kSlots packets to one destination: the rest,
        // straight from the device overflow buffer
        at::Tensor h_recv = d_recv.cpu();
        at::Tensor h_ew = S.words(0, S.L.off_ew, W).cpu();
        std::vector<int64_t> in_w(W), out_w(h_ew.data_ptr<int64_t>(), h_ew.data_ptr<int64_t>() + W);
        int64_t nin = 0;
        for (int r = 0; r < W; ++r) {
          in_w[r] = 4 * std::max<int64_t>(0, h_recv.data_ptr<int64_t>()[(size_t)r * slot] - kSlots);
          nin += in_w[r];
        }
        const int64_t nout = S.st(0).extra_total;
        at::Tensor sp_send = S.words(0, S.L.off_extra, nout), sp_recv = at::empty({nin}, dopt);
        pg->alltoall_base(sp_recv, sp_send, in_w, out_w)->wait();
        ++exchanges;
        at::Tensor off = at::tensor(std::vector<int64_t>{0, nin}, at::TensorOptions().dtype(at::kLong)).to(dopt);
        dls_launch_epoch(S.base(), S.L, 1, d_recv.data_ptr<int64_t>(), slot, 0, d_send.data_ptr<int64_t>(), 0,
                         sp_recv.data_ptr<int64_t>(), off.data_ptr<int64_t>(), nullptr, DLS_MODE_SPILL, stream);
        continue;
      }
      if (st != DLS_RUN) dls_fail(st);
      if (S.st(0).epochs == last_epochs) throw std::runtime_error("device epoch loop: no progress in a batch");
      last_epochs = S.st(0).epochs;
      b = std::min<int64_t>(2 * b, std::max<int64_t>(1, batch_max));
    }
    loop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0c).count();
  }
  const DlsState& s = S.st(0);
  py::dict d;
  d["finish_ps"] = s.finish_ps;
  d["channels"] = (uint32_t)s.g.nch;
  d["packets_sent"] = s.sent;
  d["epochs"] = s.epochs;
  d["packets"] = s.packets;
  d["exchanges"] = exchanges;
  d["polls"] = polls;
  d["loop_s"] = loop_s;
  return d;
}

// Every rank of a `starts`-rank collective in this process on the device, one
// block per rank, one epoch kernel per epoch.  The all-to-all is the
// transposition kernel, or -- with a 1-rank process group (`loopback`) -- an
// RCCL all-to-all of all ranks' send buffers, which a 1-rank group returns
// unchanged (rank d reads its slot from s at [s][d]): the per-epoch work of an
// 8-GPU run (one epoch kernel, one RCCL all-to-all, no host round trip) on one
// MI355X.  Returns every rank's finish time (== linksim_run_local's).
py::dict dev_run_local(py::dict params, const std::string& kind, int64_t nbytes, int64_t root,
                       std::vector<int64_t> starts, int64_t device, py::object loopback, int64_t batch_max) {
  c10::intrusive_ptr<c10d::ProcessGroup> pg;
  if (!loopback.is_none()) {
    pg = py::cast<c10::intrusive_ptr<c10d::ProcessGroup>>(loopback);
    if (pg->getSize() != 1) throw std::invalid_argument("dev_run_local: the loopback group must have one rank");
  }
  const int W = (int)starts.size();
  if (W < 1) throw std::invalid_argument("dev_run_local: no ranks");
  CollSpec cs;
  cs.kind = coll_kind(kind);
  cs.bytes = (uint64_t)nbytes;
  cs.root = (int32_t)root;
  const LinkParams lp = params_from(params);
  std::vector<LinkSim::Export> ex;
  for (int r = 0; r < W; ++r) ex.push_back(LinkSim(lp, cs, r, W, (uint64_t)starts[r]).export_state());
  const int slot = kHdr + 4 * kSlots;
  const int64_t n = (int64_t)W * W * slot;
  uint64_t exchanges = 0, polls = 0;
  double loop_s = 0;
  DevStates S;
  {
    py::gil_scoped_release nogil;
    // a stream of our own; work the caller queued before is finished first
    sync_stream((int)device);
    const c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromPool(false, (c10::DeviceIndex)device));
    void* stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
    S.upload(ex, W, kSlots, kHdr, (int)device);
    auto dopt = at::TensorOptions().dtype(at::kLong).device(at::kCUDA, device);
    at::Tensor t0 = at::full({1}, *std::min_element(starts.begin(), starts.end()), dopt);
    at::Tensor d_send = at::empty({n}, dopt), d_recv = at::empty({n}, dopt);
    // rank b's slot from source r: transposed [b][r] or loopback [r][b]
    const int64_t src_stride = pg ? (int64_t)W * slot : slot, rank_stride = pg ? slot : (int64_t)W * slot;
    std::vector<int64_t> all{n};
    sync_stream((int)device);
    const auto t0c = std::chrono::steady_clock::now();
    dls_launch_epoch(S.base(), S.L, W, nullptr, 0, 0, d_send.data_ptr<int64_t>(), (int64_t)W * slot, nullptr, nullptr,
                     t0.data_ptr<int64_t>(), DLS_MODE_FIRST, stream);
    auto exchange = [&] {
      if (pg)
        pg->alltoall_base(d_recv, d_send, all, all)->wait();
      else
        dls_launch_transpose(d_send.data_ptr<int64_t>(), d_recv.data_ptr<int64_t>(), W, slot, stream);
    };
    int64_t b = 1;
    uint64_t last_epochs = 0;

    for (;;) {
      auto one_epoch = [&] {
        exchange();
        dls_launch_epoch(S.base(), S.L, W, d_recv.data_ptr<int64_t>(), src_stride, rank_stride,
                         d_send.data_ptr<int64_t>(), (int64_t)W * slot, nullptr, nullptr, nullptr, DLS_MODE_NEXT,
                         stream);
      };
      for (int64_t i = 0; i < b; ++i) one_epoch();
      exchanges += (uint64_t)b;
      S.poll();
      ++polls;
      const int32_t st = S.status();
      if (st == DLS_DONE) break;
      if (st == DLS_SPILL) {
        // overflow words of every source, regrouped per destination in source order
        std::vector<std::vector<int64_t>> ew(W), xw(W);
        for (int s = 0; s < W; ++s) {
          at::Tensor e = S.words(s, S.L.off_ew, W).cpu();
          ew[s].assign(e.data_ptr<int64_t>(), e.data_ptr<int64_t>() + W);
          const int64_t nx = S.st(s).extra_total;
          if (nx) {
            at::Tensor x = S.words(s, S.L.off_extra, nx).cpu();
            xw[s].assign(x.data_ptr<int64_t>(), x.data_ptr<int64_t>() + nx);
          }
        }
        std::vector<int64_t> spill, off{0};
        for (int d = 0; d < W; ++d) {
          for (int s = 0; s < W; ++s) {
            int64_t o = 0;
            for (int dd = 0; dd < d; ++dd) o += ew[s][dd];
            spill.insert(spill.end(), xw[s].begin() + o, xw[s].begin() + o + ew[s][d]);
          }
          off.push_back((int64_t)spill.size());
        }
        if (spill.empty()) spill.push_back(0);
        at::Tensor d_sp = at::tensor(spill, at::TensorOptions().dtype(at::kLong)).to(dopt);
        at::Tensor d_off = at::tensor(off, at::TensorOptions().dtype(at::kLong)).to(dopt);
        dls_launch_epoch(S.base(), S.L, W, d_recv.data_ptr<int64_t>(), src_stride, rank_stride,
                         d_send.data_ptr<int64_t>(), (int64_t)W * slot, d_sp.data_ptr<int64_t>(),
                         d_off.data_ptr<int64_t>(), nullptr, DLS_MODE_SPILL, stream);
        sync_stream((int)device);  // d_sp / d_off are freed on return
        continue;
      }
      if (st != DLS_RUN) dls_fail(st);
      if (S.st(0).epochs == last_epochs) throw std::runtime_error("device epoch loop: no progress in a batch");
      last_epochs = S.st(0).epochs;
      b = std::min<int64_t>(2 * b, std::max<int64_t>(1, batch_max));
    }
    loop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0c).count();
  }
  std::vector<uint64_t> fin(W);
  uint64_t packets = 0;
  for (int r = 0; r < W; ++r) {
    if (S.st(r).status != DLS_DONE) dls_fail(S.st(r).status);
    fin[r] = S.st(r).finish_ps;
    packets += S.st(r).packets;
  }
  py::dict d;
  d["finish_ps"] = fin;
  d["epochs"] = S.st(0).epochs;
  d["packets"] = packets;
  d["exchanges"] = exchanges;
  d["polls"] = polls;
  d["loop_s"] = loop_s;
  d["us_per_epoch"] = loop_s * 1e6 / (double)std::max<uint64_t>(1, exchanges);
  py::list prof;  // rank 0's epoch-kernel shader clocks per launch: load, unpack, pack, store | emit, reductions, slots
  for (int i = 0; i < 7; ++i) prof.append((double)S.st(0).prof[i] / (double)std::max<uint64_t>(1, exchanges + 1));
  d["kernel_clocks_per_launch"] = prof;
  d["state_bytes_per_rank"] = (int64_t)S.L.bytes;
  return d;
}

}  // namespace asim

// ASIM_SEGV_TRACE=1: print the native stack on SIGSEGV (GPU boxes have no debugger)
static void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  if (const char* e = std::getenv("ASIM_SEGV_TRACE"); e && e[0] == '1') signal(SIGSEGV, segv_trace);
  m.doc() = "native epoch loop of the packet-level collective over a torch.distributed ProcessGroup";
  m.def("exchange_run", &asim::exchange_run, py::arg("group"), py::arg("params"), py::arg("kind"), py::arg("bytes"),
        py::arg("root"), py::arg("start_ps"), py::arg("device") = -1);
  m.def("a2a_bench", &asim::a2a_bench, py::arg("group"), py::arg("iters") = 1000, py::arg("warm") = 50,
        py::arg("device") = -1, py::arg("shape_world") = 0);
  m.def("exchange_run_device", &asim::exchange_run_device, py::arg("group"), py::arg("params"), py::arg("kind"),
        py::arg("bytes"), py::arg("root"), py::arg("start_ps"), py::arg("device"), py::arg("batch_max") = 16);
  m.def("dev_run_local", &asim::dev_run_local, py::arg("params"), py::arg("kind"), py::arg("bytes"), py::arg("root"),
        py::arg("starts"), py::arg("device"), py::arg("loopback") = py::none(), py::arg("batch_max") = 16);
}
