// Human-readable dump of the simulated pipeline (reference
// gpgpu_sim::dump_pipeline, gpu-sim.cc:2138-2179, and the `dp` gdb macro of
// .gdbinit:10-40).  Works on the engine's raw state image, so the MI355X
// engine's device-resident state is decoded on the host exactly like the CPU
// engine's.
#include <cstdio>
#include <sstream>

#include "simulator.h"

namespace asim {

static void sb_regs(std::ostringstream& o, const uint64_t* sb) {
  bool any = false;
  for (int w = 0; w < 4; ++w)
    for (int b = 0; b < 64; ++b)
      if (sb[w] >> b & 1ull) {
        o << (any ? "," : "") << "r" << (w * 64 + b - 1);
        any = true;
      }
  if (!any) o << "-";
}

std::string dump_sm_state(const SMState& s, const SimCfg& c, const TInst* const* slot_insts) {
  std::ostringstream o;
  o << "=== SM " << s.id << " @ cycle " << s.cycle << ": " << s.n_cta_active << " CTAs, "
    << s.outstanding << " packets in flight, outq " << s.outq_n << ", inq " << s.inq_n << ", L1 waiters " << s.n_pend
    << ", quiet cycles skipped " << s.skipped_cycles << "\n";
  const uint32_t nw = c.max_warps_per_sm < (uint32_t)kMaxWarps ? c.max_warps_per_sm : (uint32_t)kMaxWarps;
  for (uint32_t w = 0; w < nw; ++w) {
    const uint8_t f = s.w_flags[w];
    if (!(f & WF_ACTIVE)) continue;
    o << "  warp " << w << " cta-slot " << (int)s.w_cta[w] << " pc-index " << s.w_head[w] << "/" << s.w_end[w]
      << " ibuf " << (int)s.w_ibuf[w] << " inflight " << (int)s.w_inflight[w] << " loads " << s.w_loads[w]
      << " store-acks " << s.w_stores[w] << " flags";
    if (f & WF_EXITING) o << " EXITING";
    if (f & WF_BARRIER) o << " BARRIER";
    if (f & WF_MEMBAR) o << " MEMBAR";
    if (f & WF_WAITCNT) o << " WAITCNT";
    o << " scoreboard ";
    sb_regs(o, s.w_sb[w]);
    const TInst* insts = slot_insts[s.w_head[w] >> kSlotShift];
    if (s.w_ibuf[w] && insts) {
      const TInst& in = insts[s.w_head[w] & kIdxMask];
      o << " next " << opcode_name(in.opcode) << " pc 0x" << std::hex << in.pc << std::dec;
    }
    o << "\n";
  }
  o << "  ID_OC:";
  bool any = false;
  for (uint32_t sc = 0; sc < (uint32_t)kMaxSched; ++sc)
    for (uint32_t u = 0; u < (uint32_t)U_COUNT; ++u)
      if (s.idoc_mask >> (sc * U_COUNT + u) & 1ull) {
        const uint32_t k = sc * U_COUNT + u;
        o << " [sched " << sc << " unit " << u << " warp " << (int)(s.idoc_meta[k] & 0xff) << " "
          << opcode_name(s.idoc_inst[k].opcode) << "]";
        any = true;
      }
  o << (any ? "\n" : " empty\n") << "  operand collectors:";
  any = false;
  for (uint32_t i = 0; i < (uint32_t)kMaxOC; ++i)
    if (s.oc_mask >> i & 1u) {
      o << " [oc " << i << " warp " << (int)(s.oc_info[i] & 0xff) << " " << opcode_name(s.oc_inst[i].opcode)
        << " reads-left " << (int)((s.oc_banks[i] >> 40) & 0xff) << "]";
      any = true;
    }
  o << (any ? "\n" : " empty\n");
  if (s.ldst.busy)
    o << "  LD/ST: warp " << (int)s.ldst.warp << " " << opcode_name(s.ldst.inst.opcode) << " access "
      << (int)s.ldst.next << "/" << (int)s.ldst.inst.width << "\n";
  else
    o << "  LD/ST: idle\n";
  o << "  L1 MSHRs:";
  any = false;
  for (uint32_t i = 0; i < c.l1.mshr_entries && i < (uint32_t)kMaxL1Mshr; ++i)
    if (s.mshr[i].valid) {
      o << " [0x" << std::hex << s.mshr[i].line << std::dec << " sectors " << (int)s.mshr[i].requested << "]";
      any = true;
    }
  o << (any ? "\n" : " none\n");
  return o.str();
}

std::string dump_chan_state(const ChanState& ch, const SimCfg& c) {
  std::ostringstream o;
  o << "=== memory channel " << ch.id << ": DRAM latency pipe " << ch.lat_n << ", scheduler queue " << ch.q_n
    << ", returns " << ch.ret_n << "\n";
  for (uint32_t j = 0; j < c.n_sub_per_mem && j < (uint32_t)kMaxSubPerCh; ++j) {
    const SubPart& sp = ch.sp[j];
    uint32_t mshrs = 0;
    for (uint32_t i = 0; i < (uint32_t)kMaxL2Mshr; ++i) mshrs += sp.mshr[i].valid ? 1 : 0;
    o << "  sub-partition " << j << ": icnt->L2 " << sp.inq_n << ", ROP " << sp.rop_n << ", replies " << sp.rep_n
      << ", DRAM->L2 " << sp.fill_n << ", waiting requests " << sp.n_wait << ", L2 MSHRs " << mshrs
      << ", to DRAM " << sp.n_l2dram << ", input backlog " << sp.ovf_n << "\n";
    for (uint32_t k = 0; k < sp.rop_n && k < 4; ++k) {
      const Pkt& p = sp.rop[(sp.rop_head + k) % kRopQ];
      o << "    ROP[" << k << "] type " << (int)p.type << " line 0x" << std::hex << p.addr << std::dec
        << " sectors " << (int)p.sectors << " from SM " << p.src << " ready " << p.t / c.per_l2 << "\n";
    }
    uint32_t shown = 0;
    for (uint32_t k = 0; k < sp.n_wait && shown < 4; ++k) {
      const L2Wait& e = sp.wait[k];
      if (!e.valid) continue;
      o << "    waiter line 0x" << std::hex << e.line << std::dec << " need " << (int)e.need << " type "
        << (int)e.type << " for SM " << e.src << "\n";
      ++shown;
    }
  }
  for (uint32_t b = 0; b < c.nbk && b < (uint32_t)kMaxBanksDram; ++b)
    if (ch.bk[b].open) o << "  bank " << b << " open row " << ch.bk[b].row << "\n";
  return o.str();
}

std::string Simulator::dump_pipeline(int sm, int ch) {
  std::vector<uint8_t> img;
  eng_->snapshot(img);
  const SMState* sms = reinterpret_cast<const SMState*>(img.data());
  const ChanState* chs = reinterpret_cast<const ChanState*>(img.data() + sizeof(SMState) * cfg_.n_sm);
  std::string out;
  const TInst* slot_insts[kMaxConc] = {};
  for (int k = 0; k < kMaxConc; ++k)
    if (slot_op_[k] && slot_op_[k]->rk && !slot_op_[k]->rk->streamed() && !slot_op_[k]->rk->insts.empty()) slot_insts[k] = slot_op_[k]->rk->insts.data();
  for (uint32_t i = 0; i < cfg_.n_sm; ++i)
    if (sm == -1 || (sm >= 0 && (uint32_t)sm == i)) {
      if (sm == -1 && sms[i].n_cta_active == 0 && sms[i].outstanding == 0) continue;  // skip idle SMs in "all"
      out += dump_sm_state(sms[i], cfg_, slot_insts);
    }
  for (uint32_t i = 0; i < cfg_.n_mem; ++i)
    if (ch == -1 || (ch >= 0 && (uint32_t)ch == i)) {
      const ChanState& cs = chs[i];
      bool busy = cs.lat_n || cs.q_n || cs.ret_n;
      for (uint32_t j = 0; j < cfg_.n_sub_per_mem && j < (uint32_t)kMaxSubPerCh; ++j) {
        const SubPart& sp = cs.sp[j];
        busy = busy || sp.inq_n || sp.rop_n || sp.rep_n || sp.fill_n || sp.n_wait || sp.n_l2dram;
      }
      if (ch == -1 && !busy) continue;  // skip idle channels in "all"
      out += dump_chan_state(cs, cfg_);
    }
  return out;
}

}  // namespace asim
