// Interactive debugger of a timing simulation (reference gpgpu_sim::gpgpu_debug,
// gpu-simulator/gpgpu-sim/src/debug.cc:40-220, entered every cycle when
// g_interactive_debugger_enabled, gpu-sim.cc:1984-1990; the SIGTRAP at
// g_single_step, gpu-sim.cc:1868, 1984-1987).
//
// The reference steps its PTX functional model and watches 32-bit memory
// words.  In this trace-driven timing simulator the observable program state
// is the pipeline and the memory traffic, so:
//   * single step  = advance the whole simulated GPU by N steps of
//                    -sim_debug_step cycles (default: one PDES epoch), on
//                    either engine (the CPU engine for interactive use);
//   * breakpoint   = a warp issues the instruction at a PC (optionally on one
//                    SM, optionally only warp w), or the clock reaches a cycle;
//   * watchpoint   = a memory request for the line holding an address leaves
//                    an SM, or an L2 sub-partition looks it up;
//   * inspection   = the reference's dump_pipeline ("dp"), per-channel dumps,
//                    run statistics.
// Breakpoints and watchpoints are evaluated on the engine's debug trace
// events (EV_ISSUE, EV_PKT_SEND, EV_L2_ACCESS), which the debugger switches on.
// Commands come from stdin, or from -sim_debug_script (one per line; at the
// end of the script the run continues to completion), so a session is
// reproducible and testable.
#pragma once
#include <cstdint>
#include <functional>
#include <istream>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../model/config.h"

namespace asim {

class Debugger {
 public:
  struct Hooks {
    std::function<void(const std::string&)> print;
    std::function<std::string(int sm, int ch)> dump;  // pipeline dump (Simulator::dump_pipeline)
    std::function<std::string()> status;              // one-line run status
  };
  // `script`: command file ("" = stdin); `stop_at`: cycle to stop at first
  // (0 = stop before the first step, like the reference's single_step = true)
  Debugger(const std::string& script, uint64_t stop_at, Hooks hooks);

  // trace streams the debugger needs recorded
  static uint32_t trace_mask() { return TS_WARP_SCHEDULER | TS_INTERCONNECT | TS_MEMORY_SUBPARTITION_UNIT; }

  // after each simulated step: the events recorded in it; returns false when
  // the user quits (the run stops like at -gpgpu_max_cycle)
  bool after_step(uint64_t now, const std::vector<TraceEv>& ev, uint32_t n_sm, uint32_t l2_to_core_num,
                  uint32_t l2_to_core_den);

  // commands a session issued (tests inspect them)
  size_t commands_run() const { return ncmd_; }

 private:
  struct Bp {
    enum Kind { PC, ADDR, CYCLE } kind;
    uint64_t v;     // PC, line address, or cycle
    int sm = -1;    // PC: only this SM (-1: any)
    int warp = -1;  // PC: only this warp
    uint64_t hits = 0;
  };
  bool prompt(uint64_t now);  // command loop; false = quit
  bool next_line(std::string& line);
  void help();

  Hooks h_;
  std::unique_ptr<std::istream> file_;
  bool from_file_ = false;
  bool stepping_ = true;      // stop after every step
  uint64_t steps_left_ = 0;   // "s N": steps before the next stop
  uint64_t stop_at_ = 0;
  std::map<int, Bp> bps_;
  int next_id_ = 1;
  size_t ncmd_ = 0;
  bool quit_ = false;
};

}  // namespace asim
