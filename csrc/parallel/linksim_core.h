// Single-source core of the packet link model (linksim.h): the schedule
// geometry of one rank's collective (RCCL-style rings / chains / direct
// sends, cut into channel x step x slice packets) and the per-packet rules
// that both the host LinkSim (linksim.cc) and the device-resident epoch loop
// (linksim_dev.hip) run.  Everything here is plain data plus SIM_HD
// functions, so the two paths cannot drift apart.
#pragma once
#include <math.h>
#include <stdint.h>

#include "model/hd.h"

namespace asim {

constexpr int kLsMaxStride = 64;  // ring channels per collective (<= links, <= max_channels)
constexpr int kLsMaxLinks = 64;   // point-to-point links per simulated GPU

struct LsGeom {
  int32_t kind = 0;  // CollKind
  int32_t root = 0;
  int32_t rank = 0, world = 1;
  int32_t nch = 1, nsteps = 0;
  int32_t nlinks = 1;
  uint32_t nslices = 1;
  uint32_t slice_bytes = 131072;  // max(slice_bytes, 64)
  uint32_t pad = 0;
  uint64_t chunk = 1;  // bytes per (channel, step)
  uint64_t lat_ps = 0, epoch_ps = 0;
  double ps_per_byte_link = 0, ps_per_byte_mem = 0;
  int32_t stride[kLsMaxStride] = {};
};

// one pending send of the rank's schedule; (chan, step, slice) is unique among
// pending sends, so the order below is total and every heap pops the same way
struct LsReady {
  uint64_t t;
  int32_t chan, step, slice, pad;
};

SIM_HDI bool ls_before(const LsReady& a, const LsReady& b) {
  if (a.t != b.t) return a.t < b.t;
  if (a.chan != b.chan) return a.chan < b.chan;
  if (a.step != b.step) return a.step < b.step;
  return a.slice < b.slice;
}

// a mod n in [0, n); the operands here are almost always within one period
// (peer = rank +- stride), which skips the integer division
SIM_HDI int ls_mod(int a, int n) {
  if (a >= 0) {
    if (a < n) return a;
    if (a < 2 * n) return a - n;
  } else if (a >= -n) {
    return a + n;
  }
  const int m = a % n;
  return m < 0 ? m + n : m;
}

SIM_HDI int ls_inv_mod(int s, int n) {
  for (int x = 1; x < n; ++x)
    if ((s * x) % n == 1) return x;
  return 1;
}

// position of rank r along a chain with stride s starting after `first`
SIM_HDI int ls_chain_pos(int r, int first, int s, int N) { return ls_mod((r - first) * ls_inv_mod(s, N), N); }

// collective kinds (linksim.h CollKind)
enum : int32_t { LS_ALLREDUCE = 0, LS_ALLGATHER, LS_REDUCESCATTER, LS_BROADCAST, LS_REDUCE, LS_ALLTOALL, LS_SENDRECV };

SIM_HDI int ls_send_peer(const LsGeom& g, int ch, int k) {
  const int N = g.world, r = g.rank, s = g.stride[ch];
  if (N <= 1 || k < 0 || k >= g.nsteps) return -1;
  switch (g.kind) {
    case LS_ALLREDUCE:
    case LS_ALLGATHER:
    case LS_REDUCESCATTER: return ls_mod(r + s, N);
    case LS_BROADCAST: {
      const int pos = ls_chain_pos(r, g.root, s, N);
      return (k == pos && pos < N - 1) ? ls_mod(r + s, N) : -1;
    }
    case LS_REDUCE: {
      const int pos = ls_chain_pos(r, g.root + s, s, N);  // root is last
      return (k == pos && pos < N - 1) ? ls_mod(r + s, N) : -1;
    }
    case LS_ALLTOALL: return ls_mod(r + k + 1, N);
    case LS_SENDRECV: return ls_mod(r + 1, N);
  }
  return -1;
}

SIM_HDI int ls_recv_peer(const LsGeom& g, int ch, int k) {
  const int N = g.world, r = g.rank, s = g.stride[ch];
  if (N <= 1 || k < 0 || k >= g.nsteps) return -1;
  switch (g.kind) {
    case LS_ALLREDUCE:
    case LS_ALLGATHER:
    case LS_REDUCESCATTER: return ls_mod(r - s, N);
    case LS_BROADCAST: {
      const int pos = ls_chain_pos(r, g.root, s, N);
      return (pos > 0 && k == pos - 1) ? ls_mod(r - s, N) : -1;
    }
    case LS_REDUCE: {
      const int pos = ls_chain_pos(r, g.root + s, s, N);
      return (pos > 0 && k == pos - 1) ? ls_mod(r - s, N) : -1;
    }
    case LS_ALLTOALL: return ls_mod(r - k - 1, N);
    case LS_SENDRECV: return ls_mod(r - 1, N);
  }
  return -1;
}

SIM_HDI bool ls_recv_reduces(const LsGeom& g, int k) {
  switch (g.kind) {
    case LS_ALLREDUCE: return k < g.world - 1;
    case LS_REDUCESCATTER:
    case LS_REDUCE: return true;
    default: return false;
  }
}

// a step's arrival enables the next step's send (pipelined rings / chains)
SIM_HDI bool ls_forwards(const LsGeom& g) { return g.kind != LS_ALLTOALL && g.kind != LS_SENDRECV; }

SIM_HDI uint32_t ls_slice_len(const LsGeom& g, int s) {
  const uint64_t off = (uint64_t)s * g.slice_bytes;
  const uint64_t rest = g.chunk - off;
  return (uint32_t)(rest < g.slice_bytes ? rest : g.slice_bytes);
}

SIM_HDI int ls_link_of(const LsGeom& g, int dst) {
  const int o = ls_mod(dst - g.rank - 1, g.world);
  return o < g.nlinks ? o : o % g.nlinks;
}

// serialisation of b bytes on a link / completion of a received packet's local reduce or copy
SIM_HDI uint64_t ls_ser_ps(const LsGeom& g, uint32_t b) { return (uint64_t)ceil(b * g.ps_per_byte_link); }
SIM_HDI uint64_t ls_local_ps(const LsGeom& g, uint32_t b, int step) {
  const double per = ls_recv_reduces(g, step) ? 3.0 : 1.0;  // reduce: read mine + read recv + write
  return (uint64_t)ceil(b * per * g.ps_per_byte_mem);
}

}  // namespace asim
