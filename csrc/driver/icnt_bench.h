// Open-loop synthetic traffic through the router model (icnt_bench.cc).
#pragma once
#include <cstdint>
#include <string>

namespace asim {

struct OpenLoopParams {
  std::string traffic = "uniform";  // uniform, transpose, bitcomp, bitrev, shuffle, tornado, neighbor
  double rate = 0.1;                // offered flits per node per cycle
  uint32_t packet_flits = 1;
  uint64_t cycles = 2000, warmup = 500;
  uint64_t seed = 1;
};

struct OpenLoopResult {
  uint32_t nodes = 0;
  uint64_t packets = 0, measured_packets = 0;
  double offered = 0, accepted = 0;         // flits per node per cycle over the measurement window
  double drain_throughput = 0;              // all flits / node / cycle from the first injection to the last ejection
  double avg_latency = 0, max_latency = 0;  // creation to tail ejection, cycles
  double zero_load_latency = 0;             // the same packets' uncontended traversal
  uint32_t deadlocked = 0;
  // router activity (icnt_router.h RtAct order) and the energy of the run by
  // component (Booksim's power module role; per-event energies from the
  // .icnt file's power_* keys), pJ, and the average network power, W
  uint64_t activity[8] = {};
  double e_buffer = 0, e_xbar = 0, e_link = 0, e_alloc = 0, e_leak = 0, power_w = 0;
};

// icnt_text: a Booksim .icnt file's text (topology, router pipeline and
// microarchitecture keys)
OpenLoopResult icnt_open_loop(const std::string& icnt_text, const OpenLoopParams& p);

}  // namespace asim
