// Interactive timing debugger (see debugger.h).
#include "debugger.h"

#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>

namespace asim {

Debugger::Debugger(const std::string& script, uint64_t stop_at, Hooks hooks) : h_(std::move(hooks)), stop_at_(stop_at) {
  if (!script.empty()) {
    file_.reset(new std::ifstream(script));
    if (!*file_) throw std::runtime_error("-sim_debug_script: cannot read " + script);
    from_file_ = true;
  }
  // like the reference (single_step starts true): stop before the first step,
  // unless a stop cycle is given (g_single_step: run up to it first)
  stepping_ = stop_at == 0;
  steps_left_ = stepping_ ? 1 : 0;
}

bool Debugger::next_line(std::string& line) {
  if (from_file_) return (bool)std::getline(*file_, line);
  std::fputs("(asim debugger) ", stdout);
  std::fflush(stdout);
  return (bool)std::getline(std::cin, line);
}

void Debugger::help() {
  h_.print(
      "asim debugger commands:\n"
      "  s [n]              step n steps (default 1) of -sim_debug_step cycles\n"
      "  c                  continue to the next breakpoint / watchpoint\n"
      "  b <pc> [sm] [warp] break when a warp issues the instruction at pc (hex)\n"
      "  bc <cycle>         break when the simulation reaches a cycle\n"
      "  w <addr>           watch memory requests to the 128 B line holding addr (hex)\n"
      "  d <id>             delete a breakpoint / watchpoint\n"
      "  l                  list breakpoints and watchpoints\n"
      "  dp [sm]            dump the pipeline of an SM (default: every busy SM)\n"
      "  dm [ch]            dump a memory channel (default: every busy channel)\n"
      "  i                  run status (cycle, instructions)\n"
      "  q                  stop the simulation here\n"
      "  h                  this help\n");
}

bool Debugger::after_step(uint64_t now, const std::vector<TraceEv>& ev, uint32_t n_sm, uint32_t l2_num,
                          uint32_t l2_den) {
  if (quit_) return false;
  bool stop = false;
  char b[256];
  for (const TraceEv& e : ev)
    for (auto& kv : bps_) {
      Bp& bp = kv.second;
      bool hit = false;
      if (bp.kind == Bp::PC && e.kind == EV_ISSUE && (e.b & 0xffffffffull) == bp.v &&
          (bp.sm < 0 || e.unit == (uint32_t)bp.sm) && (bp.warp < 0 || e.a == (uint16_t)bp.warp)) {
        hit = true;
        snprintf(b, sizeof(b), "asim debugger: breakpoint %d hit: core %u warp %u issued pc 0x%llx at cycle %llu\n",
                 kv.first, e.unit, e.a, (unsigned long long)bp.v, (unsigned long long)e.cycle);
      } else if (bp.kind == Bp::ADDR && (e.b >> 7) == (bp.v >> 7)) {
        if (e.kind == EV_PKT_SEND && e.unit < n_sm) {
          hit = true;
          snprintf(b, sizeof(b),
                   "asim debugger: watchpoint %d hit: core %u sends a request for line 0x%llx (addr 0x%llx) to "
                   "sub-partition %u at cycle %llu\n",
                   kv.first, e.unit, (unsigned long long)e.b, (unsigned long long)bp.v, e.a,
                   (unsigned long long)e.cycle);
        } else if (e.kind == EV_L2_ACCESS) {
          static const char* o[] = {"hit", "miss", "mshr-hit", "write-through"};
          hit = true;
          snprintf(b, sizeof(b),
                   "asim debugger: watchpoint %d hit: channel %u sub %u L2 %s for line 0x%llx at cycle ~%llu\n",
                   kv.first, e.unit - n_sm, e.a >> 8, o[e.a & 3], (unsigned long long)e.b,
                   (unsigned long long)(l2_den ? e.cycle * l2_num / l2_den : e.cycle));
        }
      }
      if (hit) {
        ++bp.hits;
        h_.print(b);
        stop = true;
      }
    }
  for (auto& kv : bps_)
    if (kv.second.kind == Bp::CYCLE && !kv.second.hits && now >= kv.second.v) {
      ++kv.second.hits;
      snprintf(b, sizeof(b), "asim debugger: breakpoint %d hit: cycle %llu reached (now %llu)\n", kv.first,
               (unsigned long long)kv.second.v, (unsigned long long)now);
      h_.print(b);
      stop = true;
    }
  if (stop_at_ && now >= stop_at_) {
    stop_at_ = 0;
    stop = true;
  }
  if (stepping_ && steps_left_ && --steps_left_ == 0) stop = true;
  if (!stop) return true;
  stepping_ = false;
  steps_left_ = 0;
  return prompt(now);
}

bool Debugger::prompt(uint64_t now) {
  char b[160];
  snprintf(b, sizeof(b), "asim debugger: stopped at cycle %llu\n", (unsigned long long)now);
  h_.print(b);
  std::string line;
  while (next_line(line)) {
    std::istringstream is(line);
    std::string cmd;
    if (!(is >> cmd) || cmd[0] == '#') continue;
    ++ncmd_;
    h_.print("(asim debugger) " + line + "\n");
    if (cmd == "s" || cmd == "step" || cmd == "n") {
      uint64_t n = 1;
      is >> n;
      stepping_ = true;
      steps_left_ = n ? n : 1;
      return true;
    } else if (cmd == "c" || cmd == "continue") {
      stepping_ = false;
      return true;
    } else if (cmd == "b" || cmd == "break") {
      std::string pc;
      Bp bp{Bp::PC, 0};
      if (!(is >> pc)) {
        h_.print("usage: b <pc> [sm] [warp]\n");
        continue;
      }
      bp.v = std::stoull(pc, nullptr, 16);
      is >> bp.sm >> bp.warp;
      bps_[next_id_] = bp;
      snprintf(b, sizeof(b), "breakpoint %d at pc 0x%llx\n", next_id_++, (unsigned long long)bp.v);
      h_.print(b);
    } else if (cmd == "bc") {
      Bp bp{Bp::CYCLE, 0};
      if (!(is >> bp.v)) {
        h_.print("usage: bc <cycle>\n");
        continue;
      }
      bps_[next_id_] = bp;
      snprintf(b, sizeof(b), "breakpoint %d at cycle %llu\n", next_id_++, (unsigned long long)bp.v);
      h_.print(b);
    } else if (cmd == "w" || cmd == "watch") {
      std::string a;
      if (!(is >> a)) {
        h_.print("usage: w <addr>\n");
        continue;
      }
      Bp bp{Bp::ADDR, std::stoull(a, nullptr, 16)};
      bps_[next_id_] = bp;
      snprintf(b, sizeof(b), "watchpoint %d on line 0x%llx\n", next_id_++, (unsigned long long)(bp.v & ~127ull));
      h_.print(b);
    } else if (cmd == "d" || cmd == "delete") {
      int id = 0;
      is >> id;
      h_.print(bps_.erase(id) ? "deleted\n" : "no such breakpoint\n");
    } else if (cmd == "l" || cmd == "list") {
      if (bps_.empty()) h_.print("no breakpoints\n");
      for (auto& kv : bps_) {
        const Bp& p = kv.second;
        if (p.kind == Bp::PC)
          snprintf(b, sizeof(b), "%d: break pc 0x%llx sm %d warp %d (hits %llu)\n", kv.first,
                   (unsigned long long)p.v, p.sm, p.warp, (unsigned long long)p.hits);
        else if (p.kind == Bp::CYCLE)
          snprintf(b, sizeof(b), "%d: break cycle %llu (hits %llu)\n", kv.first, (unsigned long long)p.v,
                   (unsigned long long)p.hits);
        else
          snprintf(b, sizeof(b), "%d: watch line 0x%llx (hits %llu)\n", kv.first, (unsigned long long)(p.v & ~127ull),
                   (unsigned long long)p.hits);
        h_.print(b);
      }
    } else if (cmd == "dp") {
      int sm = -1;
      is >> sm;
      h_.print(h_.dump(sm, -2));
    } else if (cmd == "dm") {
      int ch = -1;
      is >> ch;
      h_.print(h_.dump(-2, ch));
    } else if (cmd == "i" || cmd == "info") {
      h_.print(h_.status() + "\n");
    } else if (cmd == "q" || cmd == "quit") {
      quit_ = true;
      h_.print("asim debugger: simulation stopped by the user\n");
      return false;
    } else if (cmd == "h" || cmd == "help") {
      help();
    } else {
      h_.print("unknown command '" + cmd + "' (h for help)\n");
    }
  }
  // end of input (script exhausted / EOF): run to completion, breakpoints off
  bps_.clear();
  stepping_ = false;
  return true;
}

}  // namespace asim
