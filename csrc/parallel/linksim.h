// Packet-level inter-GPU link model for collectives (-collective_model packet).
//
// The reference only charges a constant latency per ncclAllReduce
// (gpu-simulator/main.cc:116-122, -nccl_allreduce_latency gpu-sim.cc:760-762)
// and drops the call's arguments (tracer_tool.cu:800-819).  Here a collective
// is decomposed the way RCCL executes it -- channels of ring/chain pipelines
// (or direct all-to-all sends), each chunk cut into slices -- and every slice
// is a packet on a point-to-point xGMI link with serialisation (bytes / link
// bandwidth), link latency, per-link FIFO contention, and a local reduce/copy
// cost on the receiving GPU.
//
// Execution is a conservative parallel discrete-event simulation: one LinkSim
// per simulated GPU (= per MI355X rank).  Time advances in epochs no longer
// than the link latency, so a packet sent in an epoch can only arrive in a
// later one; after every epoch the ranks exchange the packets they emitted
// with an all-to-all (RCCL over xGMI in parallel/collectives.py).  The same
// classes run all ranks inside one process (run_local) -- the two paths are
// bit-identical, which is what the multi-process tests check.
#pragma once
#include <cstdint>
#include <queue>
#include <string>
#include <vector>

#include "linksim_core.h"

namespace asim {

struct LinkParams {
  double link_gbps = 153.0;     // per direction, per link (GB/s = bytes/ns)
  double latency_ns = 1000.0;   // per hop
  uint32_t links = 7;           // links per GPU (fully connected: one per peer when world-1 <= links)
  uint32_t slice_bytes = 131072;
  uint32_t max_channels = 16;
  double reduce_gbps = 900.0;   // local memory bandwidth used by reduce / copy
};

enum CollKind : int32_t { CK_ALLREDUCE = 0, CK_ALLGATHER, CK_REDUCESCATTER, CK_BROADCAST, CK_REDUCE, CK_ALLTOALL,
                          CK_SENDRECV };

CollKind coll_kind(const std::string& name);  // AllReduce, AllGather, ... (throws if unknown)

struct CollSpec {
  CollKind kind = CK_ALLREDUCE;
  uint64_t bytes = 0;  // buffer size (same convention as the analytic model)
  int32_t root = 0;
};

// one slice on the wire: 32 bytes, packed into 4 x int64 for the exchange
struct LinkPkt {
  int32_t src, dst;
  int32_t chan, step;
  int32_t slice;
  uint32_t bytes;
  uint64_t arrive_ps;
};
static_assert(sizeof(LinkPkt) == 32, "LinkPkt must stay 32 bytes");

class LinkSim {
 public:
  LinkSim(const LinkParams& p, const CollSpec& c, int rank, int world, uint64_t start_ps);
  // emit every packet whose send starts before t_end (appended to out)
  void emit(uint64_t t_end, std::vector<LinkPkt>& out);
  // deliver packets addressed to this rank (any order; processed deterministically)
  void receive(const LinkPkt* p, size_t n);
  // earliest time this rank has local work (UINT64_MAX if none)
  uint64_t next_event() const;
  bool done() const { return recv_left_ == 0 && send_left_ == 0; }
  uint64_t finish_ps() const { return finish_ps_; }
  uint64_t epoch_ps() const { return g_.epoch_ps; }
  uint32_t channels() const { return (uint32_t)g_.nch; }
  uint64_t packets_sent() const { return sent_; }
  int world() const { return g_.world; }

  // the whole rank state, for the device-resident epoch loop (linksim_dev.hip)
  // to take over: schedule geometry, pending sends (any order), link clocks,
  // counters
  struct Export {
    LsGeom g;
    std::vector<LsReady> ready;
    std::vector<uint64_t> link_free;
    uint64_t recv_left, send_left, sent, finish_ps;
  };
  Export export_state() const;

  // the rank's role at (channel, step): peer it sends to / receives from (-1 none)
  int send_peer(int c, int k) const;
  int recv_peer(int c, int k) const;
  bool recv_reduces(int k) const;

 private:
  struct Later {
    bool operator()(const LsReady& a, const LsReady& b) const { return ls_before(b, a); }
  };
  void push_send(uint64_t t, int c, int k, int s);

  LinkParams p_;
  LsGeom g_;
  std::priority_queue<LsReady, std::vector<LsReady>, Later> ready_;
  std::vector<uint64_t> link_free_;
  uint64_t recv_left_ = 0, send_left_ = 0, sent_ = 0;
  uint64_t finish_ps_ = 0;
};

// One epoch of the distributed packet exchange (parallel/collectives.py),
// packed and unpacked natively so the per-epoch host work is two calls around
// the all-to-all.  Fixed layout: per destination a slot of `hdr` header words
// {packets for it, this rank's largest per-destination count, announced next
// event, announced busy flag, earliest arrival among this epoch's packets}
// followed by up to `k` packets (4 int64 words each, emission order);
// packets past `k` for a destination go to `extra`, destination order.
struct EpochOut {
  std::vector<int64_t> extra;
  std::vector<int64_t> extra_words;  // per destination
  uint64_t packets = 0;
  int64_t max_count = 0;
};
void pack_epoch(LinkSim& l, uint64_t t_end, int k, int hdr, int64_t ann_next, int64_t ann_busy, int64_t* send,
                EpochOut& out);
// Deliver the received slots (+ the overflow words, source order) to `l`;
// returns {any rank busy, the earliest next event or arrival over ranks}.
struct EpochIn {
  int64_t any_busy = 0;
  int64_t next = 0;
};
EpochIn unpack_epoch(LinkSim& l, const int64_t* recv, int k, int hdr, const int64_t* extra, size_t extra_words);

// Run all `world` ranks in one process (identical results to the distributed
// driver).  start_ps[r] = when rank r reaches the collective.  Returns the
// finish time of every rank.
std::vector<uint64_t> linksim_run_local(const LinkParams& p, const CollSpec& c, const std::vector<uint64_t>& start_ps,
                                        uint64_t* epochs = nullptr, uint64_t* packets = nullptr);

}  // namespace asim
