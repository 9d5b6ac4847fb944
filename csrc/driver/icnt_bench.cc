// Open-loop synthetic-traffic runs of the router model (Booksim's standalone
// mode: reference intersim2/main.cpp + trafficmanager.cpp + traffic.cpp +
// injection.cpp).  Every node injects Bernoulli packets at `rate` flits per
// cycle towards the traffic pattern's destination for `cycles` cycles; the
// packets are simulated to their arrival in one pass of the router model
// (model/icnt_router.h), which is exact here because the whole injection
// schedule is known up front.  Latency is creation to tail ejection (source
// queueing included), accepted throughput the flits ejected during the
// measurement window [warmup, cycles) per node and cycle.
#include "icnt_bench.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <vector>

#include "../config/icnt_config.h"
#include "../model/icnt_router.h"

namespace asim {

namespace {

// splitmix64: a small deterministic generator (same stream on every host)
struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

uint32_t log2_exact(uint32_t n) {
  uint32_t b = 0;
  while ((1u << b) < n) ++b;
  if ((1u << b) != n) throw std::invalid_argument("bit-permutation traffic needs a power-of-two node count");
  return b;
}

// destination of node s under the pattern (Booksim traffic.cpp names)
uint32_t destination(const std::string& t, uint32_t s, uint32_t N, uint32_t k, uint32_t n, Rng& r) {
  if (t == "uniform") {
    for (;;) {
      const uint32_t d = (uint32_t)(r.next() % N);
      if (d != s || N == 1) return d;
    }
  }
  if (t == "bitcomp") return ~s & ((1u << log2_exact(N)) - 1);
  if (t == "transpose") {
    const uint32_t b = log2_exact(N);
    if (b % 2) throw std::invalid_argument("transpose traffic needs an even number of address bits");
    const uint32_t h = b / 2, m = (1u << h) - 1;
    return ((s & m) << h) | (s >> h);
  }
  if (t == "bitrev") {
    const uint32_t b = log2_exact(N);
    uint32_t d = 0;
    for (uint32_t i = 0; i < b; ++i) d |= ((s >> i) & 1u) << (b - 1 - i);
    return d;
  }
  if (t == "shuffle") {
    const uint32_t b = log2_exact(N);
    return ((s << 1) | (s >> (b - 1))) & (N - 1);
  }
  if (t == "tornado" || t == "neighbor") {
    // per dimension of a k-ary n-cube: half way round (tornado) or the next router
    uint32_t d = 0, pw = 1, x = s;
    for (uint32_t i = 0; i < n; ++i, pw *= k) {
      const uint32_t xi = x % k;
      const uint32_t yi = t == "tornado" ? (xi + (k + 1) / 2 - 1) % k : (xi + 1) % k;
      d += yi * pw;
      x /= k;
    }
    return d % N;
  }
  throw std::invalid_argument("unknown traffic pattern '" + t + "'");
}

// Booksim anynet network file (reference intersim2/networks/anynet.cpp
// grammar): lines "router R  router X [latency]  node n [latency] ...";
// router-router channels are bidirectional, the latency given for one
// direction (the other defaults to 1 cycle unless listed too); a node's
// latency serves its injection and ejection channels.  Links: ejection link
// n (node n's router -> node n) first, then the router-router channels.
// Routes: fewest (router delay + channel latency) by Dijkstra, ties to the
// lower router index.
struct AnyNet {
  uint32_t N = 0, R = 0, H = 1;
  std::vector<uint32_t> node_router, off, route;
  std::vector<uint16_t> lat, inj_lat;
};

AnyNet build_anynet(const std::string& text, uint32_t hop) {
  AnyNet a;
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> rr;  // (from, to) router channel -> latency
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> nodes;  // node -> (router, latency)
  std::istringstream in(text);
  std::string line;
  auto lat_of = [](std::vector<std::string>& t, size_t& i) -> uint32_t {
    if (i + 1 < t.size() && isdigit((unsigned char)t[i + 1][0])) return (uint32_t)std::stoul(t[++i]);
    return 1;
  };
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    std::vector<std::string> t;
    for (std::string x; ls >> x;) t.push_back(x);
    if (t.size() < 2 || t[0] != "router") continue;
    const uint32_t r = (uint32_t)std::stoul(t[1]);
    a.R = std::max(a.R, r + 1);
    for (size_t i = 2; i + 1 < t.size(); ++i) {
      const std::string kind = t[i];
      const uint32_t id = (uint32_t)std::stoul(t[++i]);
      const uint32_t l = lat_of(t, i);
      if (kind == "router") {
        rr[{r, id}] = l;
        a.R = std::max(a.R, id + 1);
      } else if (kind == "node") {
        nodes[id] = {r, l};
      } else {
        throw std::invalid_argument("anynet: expected 'router' or 'node', got '" + kind + "'");
      }
    }
  }
  for (auto& e : std::map<std::pair<uint32_t, uint32_t>, uint32_t>(rr))
    if (!rr.count({e.first.second, e.first.first})) rr[{e.first.second, e.first.first}] = 1;
  a.N = nodes.empty() ? 0 : nodes.rbegin()->first + 1;
  if (a.N == 0 || nodes.size() != a.N) throw std::invalid_argument("anynet: nodes must be numbered 0.. without gaps");
  a.node_router.resize(a.N);
  a.inj_lat.resize(a.N);
  a.lat.resize(a.N);
  for (auto& n : nodes) {
    a.node_router[n.first] = n.second.first;
    a.inj_lat[n.first] = a.lat[n.first] = (uint16_t)std::min<uint32_t>(n.second.second, 65535);
  }
  // router channels: link ids after the N ejection links
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> out(a.R);  // router -> (to, link)
  for (auto& e : rr) {
    out[e.first.first].push_back({e.first.second, (uint32_t)a.lat.size()});
    a.lat.push_back((uint16_t)std::min<uint32_t>(e.second, 65535));
  }
  // Dijkstra from every router (small networks: O(R^2) per source)
  std::vector<std::vector<uint32_t>> via(a.R, std::vector<uint32_t>(a.R, ~0u));  // [src][dst] -> link into dst
  for (uint32_t s0 = 0; s0 < a.R; ++s0) {
    std::vector<uint64_t> dist(a.R, ~0ull);
    std::vector<char> done(a.R, 0);
    dist[s0] = 0;
    for (uint32_t it = 0; it < a.R; ++it) {
      uint32_t u = ~0u;
      for (uint32_t x = 0; x < a.R; ++x)
        if (!done[x] && dist[x] != ~0ull && (u == ~0u || dist[x] < dist[u])) u = x;
      if (u == ~0u) break;
      done[u] = 1;
      for (auto& e : out[u]) {
        const uint64_t nd = dist[u] + hop + a.lat[e.second];
        if (nd < dist[e.first]) {
          dist[e.first] = nd;
          via[s0][e.first] = e.second;
        }
      }
    }
  }
  std::vector<uint32_t> from(a.lat.size(), 0);
  for (uint32_t r = 0; r < a.R; ++r)
    for (auto& e : out[r]) from[e.second] = r;
  a.off.assign((size_t)a.N * a.N + 1, 0);
  for (uint32_t x = 0; x < a.N; ++x)
    for (uint32_t y = 0; y < a.N; ++y) {
      const uint32_t rs = a.node_router[x], rd = a.node_router[y];
      std::vector<uint32_t> path;
      for (uint32_t r = rd; r != rs;) {
        const uint32_t l = via[rs][r];
        if (l == ~0u) throw std::invalid_argument("anynet: router " + std::to_string(rd) + " unreachable");
        path.push_back(l);
        r = from[l];
      }
      std::reverse(path.begin(), path.end());
      path.push_back(y);  // the ejection link into node y
      a.route.insert(a.route.end(), path.begin(), path.end());
      a.off[(size_t)x * a.N + y + 1] = (uint32_t)a.route.size();
      a.H = std::max<uint32_t>(a.H, (uint32_t)path.size());
    }
  return a;
}

}  // namespace

OpenLoopResult icnt_open_loop(const std::string& icnt_text, const OpenLoopParams& prm) {
  SimCfg c{};
  c.flit_size = 32;
  const auto kv = parse_booksim_config(icnt_text);
  const bool anynet = kv.count("topology") && kv.at("topology") == "anynet";
  AnyNet an;
  uint64_t nodes = 0;
  if (anynet) {
    // the router microarchitecture and pipeline from the file, the network
    // from its network_file
    auto k2 = kv;
    k2["topology"] = "fly";
    k2["k"] = "2";
    k2["n"] = "1";
    apply_topology(c, k2);
    if (!kv.count("network_file")) throw std::invalid_argument("anynet needs network_file");
    std::ifstream f(kv.at("network_file"));
    if (!f.good()) throw std::invalid_argument("cannot open anynet network_file '" + kv.at("network_file") + "'");
    std::stringstream ss;
    ss << f.rdbuf();
    an = build_anynet(ss.str(), c.hop_icnt);
    nodes = an.N;
  } else {
    nodes = apply_topology(c, kv);
  }
  if (c.rt_alloc == 0xff) throw std::invalid_argument("sw_allocator not modelled");
  c.link_contention = 2;
  if (nodes > (1u << 20)) throw std::invalid_argument("topology too large");
  const uint32_t N = (uint32_t)nodes;
  const uint32_t pf = prm.packet_flits ? prm.packet_flits : 1;
  if (prm.rate < 0 || prm.rate > 1) throw std::invalid_argument("rate must be 0..1 flits per node per cycle");
  if (prm.warmup >= prm.cycles) throw std::invalid_argument("warmup must be shorter than the run");
  // the injection schedule
  Rng r{prm.seed * 0x2545f4914f6cdd1dull + 1};
  std::vector<uint32_t> src, dst;
  std::vector<uint64_t> tinj;
  const double p_pkt = prm.rate / pf;
  for (uint64_t t = 0; t < prm.cycles; ++t)
    for (uint32_t s = 0; s < N; ++s)
      if (r.uniform() < p_pkt) {
        const uint32_t d = destination(prm.traffic, s, N, anynet ? N : c.topo_k, anynet ? 1u : c.topo_n, r);
        if (d == s) continue;  // a fixed point of a permutation sends nothing
        src.push_back(s);
        dst.push_back(d);
        tinj.push_back(t);
      }
  const uint64_t np64 = src.size();
  if (np64 > 50'000'000ull) throw std::invalid_argument("too many packets for one pass");
  const uint32_t np = (uint32_t)np64;
  RtDims d = rt_dims(c, np ? np : 1, pf);
  if (anynet) {
    d.N = an.N;
    d.L = (uint32_t)an.lat.size();
    d.U = d.N + d.L;
    d.H = an.H;
  }
  std::vector<uint64_t> st(rt_state_words(d), 0);
  std::vector<uint32_t> scratch(rt_carve(d, nullptr, nullptr), 0);
  RtWork w;
  rt_carve(d, scratch.data(), &w);
  if (anynet) {
    w.rt_off = an.off.data();
    w.rt_links = an.route.data();
    w.lat = an.lat.data();
    w.inj_lat = an.inj_lat.data();
  }
  for (uint32_t i = 0; i < np; ++i) {
    w.src[i] = src[i];
    w.dst[i] = dst[i];
    w.nfl[i] = pf;
    w.tinj[i] = tinj[i];
  }
  OpenLoopResult res;
  res.nodes = N;
  res.packets = np;
  uint64_t act[RT_ACT_COUNT] = {};
  res.deadlocked = np ? rt_simulate(c, d, st.data(), w, np, act) : 0;
  for (int i = 0; i < RT_ACT_COUNT; ++i) res.activity[i] = act[i];
  double lat = 0, zero = 0;
  uint64_t meas = 0, ejected = 0, last = 0;
  for (uint32_t i = 0; i < np; ++i) {
    const uint64_t a = w.tarr[i];
    last = std::max(last, a);
    if (a >= prm.warmup && a < prm.cycles) ejected += pf;
    if (tinj[i] >= prm.warmup) {
      lat += (double)(a - tinj[i]);
      if (anynet) {
        // injection channel + per router its delay and its output channel
        uint64_t z = an.inj_lat[src[i]] + (pf - 1);
        const size_t pr = (size_t)src[i] * an.N + dst[i];
        for (uint32_t k = an.off[pr]; k < an.off[pr + 1]; ++k) z += c.hop_icnt + an.lat[an.route[k]];
        zero += (double)z;
      } else {
        zero += (double)rt_uncontended(c, icnt_routers(c, src[i], dst[i]), pf);
      }
      ++meas;
      res.max_latency = std::max<double>(res.max_latency, (double)(a - tinj[i]));
    }
  }
  const double window = (double)(prm.cycles - prm.warmup) * N;
  res.offered = (double)meas * pf / window;
  res.accepted = (double)ejected / window;
  res.avg_latency = meas ? lat / meas : 0;
  res.zero_load_latency = meas ? zero / meas : 0;
  res.measured_packets = meas;
  // above saturation the window sees the network before its queues settle;
  // the drain rate is the bottleneck's (open loop, every packet delivered)
  res.drain_throughput = np && last ? (double)np * pf / ((double)N * (double)(last + 1)) : 0;
  // network energy from the activity (Booksim power_module.cpp's terms:
  // input buffers, crossbar, channels, allocators, buffer leakage); the
  // per-event energies are .icnt keys with ~22 nm Orion-class defaults
  auto num = [&](const char* k, double dflt) {
    auto it = kv.find(k);
    return it == kv.end() ? dflt : strtod(it->second.c_str(), nullptr);
  };
  const double bits = 8.0 * c.flit_size;
  res.e_buffer = num("power_buffer_pj_per_bit", 0.08) * bits * (double)(act[RT_ACT_BUF_WRITE] + act[RT_ACT_BUF_READ]);
  res.e_xbar = num("power_xbar_pj_per_bit", 0.06) * bits * (double)act[RT_ACT_BUF_READ];
  res.e_link = num("power_link_pj_per_bit_mm", 0.15) * num("power_link_mm", 1.0) * bits *
               (double)(act[RT_ACT_LINK] + act[RT_ACT_EJECT]);
  res.e_alloc = num("power_alloc_pj_per_request", 0.5) * (double)act[RT_ACT_SA_REQ];
  const double ghz = num("power_clock_ghz", 1.0), t_ns = (double)(last + 1) / ghz;
  // leakage: uW per buffered flit slot of every input VC
  res.e_leak = num("power_buffer_leak_uw_per_flit", 0.5) * 1e-6 * (double)d.U * d.V * d.B * t_ns * 1e3;
  const double e = res.e_buffer + res.e_xbar + res.e_link + res.e_alloc + res.e_leak;
  res.power_w = t_ns > 0 ? e * 1e-12 / (t_ns * 1e-9) : 0;
  return res;
}

}  // namespace asim
