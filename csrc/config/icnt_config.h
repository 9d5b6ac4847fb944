// Interconnect configuration files of -network_mode 1 (Booksim/intersim2
// `.icnt` files, reference gpu-simulator/gpgpu-sim/src/intersim2/
// config_utils.cpp + booksim_config.cpp grammar: `key = value;`, // and /* */
// comments, `{...}` list values).
#pragma once
#include <map>
#include <string>

#include "../model/config.h"

namespace asim {

// key -> raw value text (lists keep their braces)
std::map<std::string, std::string> parse_booksim_config(const std::string& text);

// Fill the topology fields of `c` (topo, topo_k/n/conc, hop/chan latency,
// flit size) from an .icnt file and derive the lookahead (c.icnt_latency) as
// the smallest SM<->sub-partition latency.  Clocks and the SM / sub-partition
// counts of `c` must already be set.  Throws OptionError on bad files.
void apply_intersim_config(SimCfg& c, const std::string& path);

// topology, router pipeline, flit size and router microarchitecture of a
// parsed .icnt file (icnt_mode = 1); returns the topology's node count
uint64_t apply_topology(SimCfg& c, const std::map<std::string, std::string>& kv);

// the router microarchitecture fields (rt_*) from a parsed .icnt file
void apply_router_params(SimCfg& c, const std::map<std::string, std::string>& kv);

}  // namespace asim
