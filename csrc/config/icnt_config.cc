// -network_mode 1: read a Booksim-format .icnt file and turn it into the
// per-pair latency model of the epoch engine (model/config.h icnt_pkt_lat_fs).
//
// What is kept from the reference's intersim2 network (interconnect_interface
// .cpp, networks/*, routers/iq_router.cpp): the topology (fly, mesh, torus,
// cmesh, fattree/tree4/qtree, flatfly/dragonfly), the node numbering (shader
// clusters first, then memory sub-partitions: icnt_wrapper.cc), the router
// pipeline depth (routing + VC allocation + switch allocation + traversal)
// and channel latency per hop, and the flit size used for serialisation.
// Contention is modelled at the injection and ejection ports of every node
// (as for the local crossbar); -icnt_link_contention 1 adds link
// reservations inside multi-hop topologies (icnt_links.h) and 2 the router
// microarchitecture: virtual channels, credits, the switch allocator
// (model/icnt_router.h), from num_vcs, vc_buf_size, alloc_iters,
// credit_delay, sw_allocator, sw_alloc_delay and internal_speedup.
#include "icnt_config.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "options.h"
#include "../model/icnt_router.h"

namespace asim {

std::map<std::string, std::string> parse_booksim_config(const std::string& text0) {
  // strip comments
  std::string t;
  t.reserve(text0.size());
  for (size_t i = 0; i < text0.size();) {
    if (text0.compare(i, 2, "//") == 0) {
      while (i < text0.size() && text0[i] != '\n') ++i;
    } else if (text0.compare(i, 2, "/*") == 0) {
      size_t e = text0.find("*/", i + 2);
      i = e == std::string::npos ? text0.size() : e + 2;
    } else {
      t += text0[i++];
    }
  }
  std::map<std::string, std::string> kv;
  size_t i = 0;
  while (i < t.size()) {
    size_t eq = t.find('=', i);
    if (eq == std::string::npos) break;
    std::string key = t.substr(i, eq - i);
    // value runs to the ';' at brace depth 0
    size_t j = eq + 1;
    int depth = 0;
    while (j < t.size() && !(t[j] == ';' && depth == 0)) {
      if (t[j] == '{') ++depth;
      if (t[j] == '}') --depth;
      ++j;
    }
    std::string val = t.substr(eq + 1, j - eq - 1);
    auto trim = [](std::string s) {
      size_t a = 0, b = s.size();
      while (a < b && isspace((unsigned char)s[a])) ++a;
      while (b > a && isspace((unsigned char)s[b - 1])) --b;
      return s.substr(a, b - a);
    };
    key = trim(key);
    if (!key.empty()) kv[key] = trim(val);
    i = j + 1;
  }
  return kv;
}

static long geti(const std::map<std::string, std::string>& kv, const char* k, long dflt) {
  auto it = kv.find(k);
  if (it == kv.end() || it->second.empty()) return dflt;
  char* end = nullptr;
  double v = strtod(it->second.c_str(), &end);
  if (end == it->second.c_str()) throw OptionError(std::string("interconnect config: bad value for ") + k);
  return (long)v;
}

void apply_router_params(SimCfg& c, const std::map<std::string, std::string>& kv) {
  const long vcs = geti(kv, "num_vcs", 1), buf = geti(kv, "vc_buf_size", 8), iters = geti(kv, "alloc_iters", 1);
  const long cd = geti(kv, "credit_delay", 0), sa = geti(kv, "sw_alloc_delay", 1);
  if (vcs < 1 || vcs > 64) throw OptionError("interconnect config: num_vcs must be 1..64");
  if (buf < 1 || buf > 4096) throw OptionError("interconnect config: vc_buf_size must be 1..4096");
  if (iters < 1 || iters > 16) throw OptionError("interconnect config: alloc_iters must be 1..16");
  if (cd < 0 || cd > 255 || sa < 0 || sa > 255) throw OptionError("interconnect config: credit / allocation delay out of range");
  // the injection queue's capacity in flits (interconnect_interface.cpp:129-133:
  // input_buffer_size, 9 when unset)
  const long ib = geti(kv, "input_buffer_size", 0);
  if (ib < 0 || ib > 65535) throw OptionError("interconnect config: input_buffer_size out of range");
  c.rt_inbuf = (uint16_t)(ib ? ib : 9);
  c.rt_vcs = (uint8_t)vcs;
  c.rt_buf = (uint16_t)buf;
  c.rt_iters = (uint8_t)iters;
  c.rt_credit = (uint8_t)cd;
  c.rt_sa = (uint8_t)sa;
  double sp = 1.0;
  if (kv.count("internal_speedup")) sp = strtod(kv.at("internal_speedup").c_str(), nullptr);
  if (!(sp >= 1.0 && sp <= 8.0)) throw OptionError("interconnect config: internal_speedup must be 1..8");
  c.rt_speedup_q8 = (uint16_t)(sp * 256.0 + 0.5);
  // minimal adaptive routing with a dimension-order escape VC (Booksim
  // min_adapt; meshes with >= 2 VCs), Valiant's randomised two-phase routing
  // (valiant; meshes with >= 2 VCs), else the topology's deterministic route
  const std::string rf = kv.count("routing_function") ? kv.at("routing_function") : "";
  c.rt_route = (rf == "min_adapt" || rf == "adaptive") ? 1 : (rf == "valiant") ? 2 : 0;
  const std::string al = kv.count("sw_allocator") ? kv.at("sw_allocator") : "islip";
  if (al == "islip") {
    c.rt_alloc = RT_ISLIP;
  } else if (al == "separable_input_first") {
    c.rt_alloc = RT_SEP_INPUT_FIRST;
  } else if (al == "separable_output_first") {
    c.rt_alloc = RT_SEP_OUTPUT_FIRST;
  } else if (al == "wavefront" || al == "rr_wavefront") {
    c.rt_alloc = RT_WAVEFRONT;
  } else if (al == "max_size") {
    c.rt_alloc = RT_MAX_SIZE;
  } else if (al == "pim") {
    c.rt_alloc = RT_PIM;
  } else if (al == "loa") {
    c.rt_alloc = RT_LOA;
  } else {
    c.rt_alloc = 0xff;  // refused only when the router model is on (-icnt_link_contention 2)
  }
}

uint64_t apply_topology(SimCfg& c, const std::map<std::string, std::string>& kv0) {
  auto kv = kv0;
  std::string topo = kv.count("topology") ? kv["topology"] : "mesh";
  const long k = geti(kv, "k", 8), n = geti(kv, "n", 2);
  if (k < 1 || n < 1 || k > 65535 || n > 255) throw OptionError("interconnect config: k/n out of range");
  c.topo_k = (uint16_t)k;
  c.topo_n = (uint8_t)n;
  c.topo_conc = (uint16_t)std::max<long>(1, geti(kv, "c", 1));
  uint64_t nodes = 1;
  for (long d = 0; d < n; ++d) nodes *= (uint64_t)k;
  if (topo == "fly") {
    c.topo = TOPO_FLY;
  } else if (topo == "mesh") {
    c.topo = TOPO_MESH;
  } else if (topo == "torus" || topo == "kncube") {
    c.topo = TOPO_TORUS;
  } else if (topo == "cmesh") {
    c.topo = TOPO_CMESH;
    nodes *= c.topo_conc;
  } else if (topo == "fattree" || topo == "tree4" || topo == "qtree") {
    c.topo = TOPO_FATTREE;
    if (topo == "tree4") c.topo_k = 4;
  } else if (topo == "flatfly" || topo == "dragonfly") {
    c.topo = TOPO_FLATFLY;  // one hop per differing dimension (minimal routing)
    nodes *= c.topo_conc;   // flatfly_onchip: c terminals per router
  } else {
    throw OptionError("interconnect config: unsupported topology '" + topo + "' (anynet needs a network file)");
  }
  // iq_router pipeline: routing, VC allocation, switch allocation, traversal
  const long hop = geti(kv, "routing_delay", 0) + geti(kv, "vc_alloc_delay", 1) + geti(kv, "sw_alloc_delay", 1) + 1;
  c.hop_icnt = (uint16_t)std::max<long>(1, hop);
  c.chan_icnt = (uint16_t)std::max<long>(1, geti(kv, "channel_latency", 1));
  if (kv.count("flit_size")) c.flit_size = (uint32_t)std::max<long>(8, geti(kv, "flit_size", 32));
  apply_router_params(c, kv);
  c.icnt_mode = 1;
  return nodes;
}

void apply_intersim_config(SimCfg& c, const std::string& path) {
  std::ifstream f(path);
  if (!f.good()) throw OptionError("cannot open interconnect config file '" + path + "'");
  std::stringstream ss;
  ss << f.rdbuf();
  const uint64_t nodes = apply_topology(c, parse_booksim_config(ss.str()));
  const uint64_t need = (uint64_t)c.n_clusters + c.n_subpart;
  if (nodes < need)
    throw OptionError("interconnect config: topology has " + std::to_string(nodes) + " nodes, need " +
                      std::to_string(need) + " (clusters + memory sub-partitions)");
  // lookahead = smallest pair latency in whole core cycles (>= 1, <= kMaxEpoch)
  uint64_t lo = ~0ull;
  c.icnt_latency = 1;  // icnt_pkt_lat_fs clamps to it; 1 core cycle is the floor
  for (uint32_t s = 0; s < c.n_sm; s += (c.cores_per_cluster ? c.cores_per_cluster : 1))
    for (uint32_t d = 0; d < c.n_subpart; ++d) lo = std::min(lo, icnt_pkt_lat_fs(c, s, d));
  uint64_t e = lo / c.per_core;
  if (e < 1) e = 1;
  if (e > (uint64_t)kMaxEpoch) e = (uint64_t)kMaxEpoch;
  c.icnt_latency = (uint32_t)e;
}

}  // namespace asim
