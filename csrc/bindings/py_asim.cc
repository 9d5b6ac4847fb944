// Python bindings of the native simulator (module: accel_sim_framework_distributed_amd._asim).
#include <chrono>
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../config/icnt_config.h"
#include "../driver/icnt_bench.h"
#include "../driver/simulator.h"

namespace py = pybind11;
using namespace asim;
static const size_t kLinkPktBytes = sizeof(LinkPkt);

namespace {

py::dict link_dict(const LinkParams& p) {
  py::dict d;
  d["link_gbps"] = p.link_gbps;
  d["latency_ns"] = p.latency_ns;
  d["links"] = p.links;
  d["slice_bytes"] = p.slice_bytes;
  d["max_channels"] = p.max_channels;
  d["reduce_gbps"] = p.reduce_gbps;
  return d;
}

LinkParams link_from(const py::dict& d) {
  LinkParams p;
  if (d.contains("link_gbps")) p.link_gbps = d["link_gbps"].cast<double>();
  if (d.contains("latency_ns")) p.latency_ns = d["latency_ns"].cast<double>();
  if (d.contains("links")) p.links = d["links"].cast<uint32_t>();
  if (d.contains("slice_bytes")) p.slice_bytes = d["slice_bytes"].cast<uint32_t>();
  if (d.contains("max_channels")) p.max_channels = d["max_channels"].cast<uint32_t>();
  if (d.contains("reduce_gbps")) p.reduce_gbps = d["reduce_gbps"].cast<double>();
  return p;
}

CollSpec coll_from(const std::string& kind, uint64_t bytes, int root) {
  CollSpec c;
  c.kind = coll_kind(kind);
  c.bytes = bytes;
  c.root = root;
  return c;
}

py::dict cfg_dict(const SimCfg& c) {
  py::dict d;
  d["n_sm"] = c.n_sm;
  d["n_clusters"] = c.n_clusters;
  d["n_mem"] = c.n_mem;
  d["n_sub_per_mem"] = c.n_sub_per_mem;
  d["n_subpart"] = c.n_subpart;
  d["warp_size"] = c.warp_size;
  d["max_warps_per_sm"] = c.max_warps_per_sm;
  d["max_cta_per_sm"] = c.max_cta_per_sm;
  d["n_sched"] = c.n_sched;
  d["sched_policy"] = c.sched_policy;
  d["sched_param"] = c.sched_param;
  d["max_issue_per_warp"] = c.max_issue_per_warp;
  d["dual_issue_diff"] = c.dual_issue_diff;
  d["fetch_throughput"] = c.fetch_throughput;
  d["ex_wb_width"] = c.ex_wb_width;
  d["oc_units"] = c.oc_units;
  d["reg_banks"] = c.reg_banks;
  d["l1_sets"] = c.l1.nsets;
  d["l1_assoc"] = c.l1.assoc;
  d["l1_latency"] = c.l1_latency;
  d["l1_mshr"] = c.l1.mshr_entries;
  d["l2_sets"] = c.l2.nsets;
  d["l2_assoc"] = c.l2.assoc;
  d["l2_set_index"] = c.l2.set_index;
  d["rop_latency"] = c.rop_latency;
  d["dram_latency"] = c.dram_latency;
  d["nbk"] = c.nbk;
  d["nbkgrp"] = c.nbkgrp;
  d["tRCD"] = c.tRCD;
  d["tRAS"] = c.tRAS;
  d["tRP"] = c.tRP;
  d["tRC"] = c.tRC;
  d["CL"] = c.CL;
  d["WL"] = c.WL;
  d["tCCDL"] = c.tCCDL;
  d["tRTPL"] = c.tRTPL;
  d["BL"] = c.BL;
  d["busW"] = c.busW;
  d["atom_size"] = c.atom_size;
  d["icnt_latency"] = c.icnt_latency;
  d["flit_size"] = c.flit_size;
  d["per_core_fs"] = c.per_core;
  d["per_dram_fs"] = c.per_dram;
  d["part_index"] = c.part_index;
  d["addr_chip_s"] = c.addr_chip_s;
  py::list masks;
  for (int i = 0; i < AF_COUNT; ++i) masks.append(c.addr_mask[i]);
  d["addr_mask"] = masks;
  d["sub_id_mask"] = c.sub_id_mask;
  py::list lat, ii;
  for (int i = 0; i < OC_COUNT; ++i) {
    lat.append(c.lat[i]);
    ii.append(c.ii[i]);
  }
  d["lat"] = lat;
  d["ii"] = ii;
  py::list units;
  for (int i = 0; i < U_COUNT; ++i) units.append(c.unit_count[i]);
  d["unit_count"] = units;
  d["kernel_launch_latency"] = c.kernel_launch_latency;
  d["eject_buf"] = c.eject_buf;
  d["ldst_resp_buf"] = c.ldst_resp_buf;
  d["icnt_in_pkts"] = c.icnt_in_pkts;
  d["icnt_out_limit"] = c.icnt_out_limit;
  return d;
}

SimCfg cfg_from_args(const std::vector<std::string>& args) {
  OptionRegistry r;
  register_sim_options(r);
  r.parse_cmdline(args, false);
  return derive_sim_cfg(r);
}

py::dict kernel_dict(const KernelResult& k) {
  py::dict d;
  d["name"] = k.name;
  d["uid"] = k.uid;
  d["start_cycle"] = k.start_cycle;
  d["cycles"] = k.cycles;
  d["insn"] = k.insn;
  d["warp_insn"] = k.warp_insn;
  d["n_cta"] = k.n_cta;
  d["cta_per_sm"] = k.cta_per_sm;
  d["ipc"] = k.ipc;
  d["occupancy"] = k.occupancy;
  d["wall_s"] = k.wall_s;
  d["deadlock"] = k.deadlock;
  d["avg_power_w"] = k.avg_power_w;
  d["epochs"] = k.epochs;
  return d;
}

}  // namespace

PYBIND11_MODULE(_asim, m) {
  m.doc() = "MI355X-native trace-driven GPU simulator (native core)";
  m.attr("sizeof_SMState") = sizeof(SMState);
  m.attr("sizeof_ChanState") = sizeof(ChanState);
  m.attr("offsetof_SMState_skipped") = offsetof(SMState, skipped_cycles);
  // (offset, bytes) of the fields whose contents depend on which epochs ran
  // (gather scratch, the mailbox-parity flags): compare snapshots of runs
  // with different epoch sequences (event skipping on / off) without them
  m.attr("epoch_dependent_SMState") = std::vector<std::pair<size_t, size_t>>{
      {offsetof(SMState, skey), sizeof(SMState::skey)}, {offsetof(SMState, sref), sizeof(SMState::sref)},
      {offsetof(SMState, srank), sizeof(SMState::srank)}, {offsetof(SMState, pub_nz), sizeof(SMState::pub_nz)},
      {offsetof(SMState, skipped_cycles), sizeof(SMState::skipped_cycles)}};
  m.attr("epoch_dependent_ChanState") = std::vector<std::pair<size_t, size_t>>{
      {offsetof(ChanState, skey), sizeof(ChanState::skey)}, {offsetof(ChanState, sref), sizeof(ChanState::sref)},
      {offsetof(ChanState, srank), sizeof(ChanState::srank)}, {offsetof(ChanState, pub_nz), sizeof(ChanState::pub_nz)}};
  m.attr("sizeof_TInst") = sizeof(TInst);

  m.def("gpu_available", &gpu_engine_available, "True if a HIP device is usable by the GPU engine");
  // compile-time capacities of the cycle model (per SM / per memory sub-partition)
  {
    py::dict lim;
    lim["max_warps"] = kMaxWarps;
    lim["max_cta"] = kMaxCta;
    lim["l1_lines"] = kMaxL1Lines;
    lim["l1_mshr"] = kMaxL1Mshr;
    lim["l2_lines_per_channel"] = kMaxL2LinesCh;
    lim["l2_mshr"] = kMaxL2Mshr;
    lim["sm_total"] = kMaxSmTot;
    lim["sub_total"] = kMaxSubTot;
    m.attr("limits") = lim;
  }
  m.def("gpu_cu_count", &gpu_cu_count, "compute units of the current HIP device");
  m.def("gpu_pool_stats", &gpu_pool_stats, "GPU engine caching allocator: cached bytes, caps, trims");
  m.def("gpu_engine_modes", &gpu_engine_modes, "per GPU-engine build (lds / global / split): LDS bytes, blocks per CU, registers");
  m.def("gpu_batch_stats", &gpu_batch_stats, "global-state batch launches: batches, launches, blocks per CU");
  m.def("gpu_pool_trim", &gpu_pool_trim, "give the GPU engine allocator's cached blocks back to the driver");
  m.def("gpu_cus_per_sim", &gpu_cus_per_sim, "CUs one GPU-engine simulation of this shape reserves (ASIM_GPU_STATE)");
  m.def("gpu_engine_kernel_info", []() {
    const EngineKernelInfo k = gpu_engine_kernel_info();
    py::dict d;
    if (!k.valid) return d;
    d["vgprs_per_lane"] = k.num_regs;
    d["scratch_bytes_per_lane"] = k.local_bytes;
    d["lds_static"] = k.shared_static;
    d["lds_dynamic"] = k.lds_dynamic;
    d["max_threads_per_block"] = k.max_threads;
    d["binary_version"] = k.binary_version;
    d["sm_state_bytes"] = k.sm_state_bytes;
    d["chan_state_bytes"] = k.chan_state_bytes;
    return d;
  }, "compiled resources of the persistent HIP engine kernel (needs a GPU)");
  m.def("option_names", []() {
    OptionRegistry r;
    register_sim_options(r);
    return r.names();
  });
  m.def("unmodelled_option_warnings", [](const std::vector<std::string>& args) {
    OptionRegistry r;
    register_sim_options(r);
    r.parse_cmdline(args, false);
    return unmodelled_option_warnings(r);
  }, "warnings for options that are accepted but have no effect");
  m.def("parse_config", [](const std::vector<std::string>& args) { return cfg_dict(cfg_from_args(args)); },
        "derive the model configuration from accel-sim style arguments");
  m.def("addr_decode", [](const std::vector<std::string>& args, uint64_t addr) {
    SimCfg c = cfg_from_args(args);
    AddrTlx t = addr_decode(c, addr);
    py::dict d;
    d["chip"] = t.chip;
    d["bk"] = t.bk;
    d["row"] = t.row;
    d["col"] = t.col;
    d["burst"] = t.burst;
    d["sub"] = t.sub;
    return d;
  });
  m.def("icnt_latency", [](const std::vector<std::string>& args, uint32_t sm, uint32_t sub) {
    // (packet latency SM sm <-> sub-partition sub in core cycles, lookahead in core cycles, routers)
    SimCfg c = cfg_from_args(args);
    const uint32_t node = sm / (c.cores_per_cluster ? c.cores_per_cluster : 1);
    return py::make_tuple((double)icnt_pkt_lat_fs(c, sm, sub) / (double)c.per_core, c.icnt_latency,
                          c.icnt_mode == 1 ? icnt_routers(c, node, c.n_clusters + sub) : 1u);
  }, "interconnect latency model (-network_mode 1 topology or local crossbar)");
  m.def("parse_booksim_config", [](const std::string& text) { return parse_booksim_config(text); });
  m.def(
      "icnt_path",
      [](const std::vector<std::string>& args, uint32_t a, uint32_t b) {
        // (links of the route from node a to node b, the topology's link count)
        SimCfg c = cfg_from_args(args);
        const uint64_t n = icnt_link_count(c);
        std::vector<uint32_t> v;
        if (n) icnt_route(c, a, b, [&](uint32_t l) { v.push_back(l); });
        return py::make_tuple(v, n);
      },
      "link-contention route model (icnt_links.h): interconnect nodes are clusters, then sub-partitions");
  m.def(
      "icnt_open_loop",
      [](const std::string& icnt_text, const std::string& traffic, double rate, uint32_t packet_flits,
         uint64_t cycles, uint64_t warmup, uint64_t seed) {
        OpenLoopParams p;
        p.traffic = traffic;
        p.rate = rate;
        p.packet_flits = packet_flits;
        p.cycles = cycles;
        p.warmup = warmup;
        p.seed = seed;
        OpenLoopResult r;
        {
          py::gil_scoped_release nogil;
          r = icnt_open_loop(icnt_text, p);
        }
        py::dict d;
        d["nodes"] = r.nodes;
        d["packets"] = r.packets;
        d["measured_packets"] = r.measured_packets;
        d["offered"] = r.offered;
        d["accepted"] = r.accepted;
        d["drain_throughput"] = r.drain_throughput;
        d["avg_latency"] = r.avg_latency;
        d["max_latency"] = r.max_latency;
        d["zero_load_latency"] = r.zero_load_latency;
        d["deadlocked"] = r.deadlocked;
        py::dict a;
        const char* an[] = {"buffer_writes", "buffer_reads", "link_flits", "eject_flits", "sa_requests", "credits",
                            "switch_passes"};
        for (int i = 0; i < 7; ++i) a[an[i]] = r.activity[i];
        d["activity"] = a;
        py::dict e;
        e["buffer"] = r.e_buffer;
        e["crossbar"] = r.e_xbar;
        e["link"] = r.e_link;
        e["allocator"] = r.e_alloc;
        e["leakage"] = r.e_leak;
        d["energy_pj"] = e;
        d["power_w"] = r.power_w;
        return d;
      },
      py::arg("icnt_text"), py::arg("traffic") = "uniform", py::arg("rate") = 0.1, py::arg("packet_flits") = 1,
      py::arg("cycles") = 2000, py::arg("warmup") = 500, py::arg("seed") = 1,
      "open-loop synthetic traffic through the router model (Booksim standalone mode, icnt_router.h)");
  m.def(
      "arch_energy",
      [](const std::vector<std::string>& args, double node_nm, double vdd, double dram_pj_per_bit,
         double tensor_macs_per_lane) {
        SimCfg c = cfg_from_args(args);
        ArchEnergyParams p;
        p.node_nm = node_nm;
        p.vdd = vdd;
        p.dram_pj_per_bit = dram_pj_per_bit;
        p.tensor_macs_per_lane = tensor_macs_per_lane;
        const ArchEnergy e = arch_energy(c, p);
        py::dict d, base, arrays;
        for (int i = 0; i < PA_COUNT; ++i) base[kPwrActName[i]] = e.base_nj[i];
        for (const auto& a : e.arrays) {
          py::dict x;
          x["read_nj"] = a.e_read_nj;
          x["write_nj"] = a.e_write_nj;
          x["tag_nj"] = a.e_tag_nj;
          x["leak_w"] = a.leak_w;
          x["area_mm2"] = a.area_mm2;
          x["org"] = py::make_tuple(a.ndwl, a.ndbl, a.nspd, a.sub_rows, a.sub_cols);
          arrays[py::str(a.name)] = x;
        }
        d["base_nj"] = base;
        d["arrays"] = arrays;
        d["die_mm2"] = e.die_mm2;
        d["sm_area_mm2"] = e.sm_area_mm2;
        d["leak_sm_w"] = e.leak_sm_w;
        d["leak_l2_w"] = e.leak_l2_w;
        d["vdd"] = e.tech.vdd;
        d["report"] = arch_energy_report(e);
        return d;
      },
      py::arg("args"), py::arg("node_nm") = 12.0, py::arg("vdd") = 0.0, py::arg("dram_pj_per_bit") = 3.9,
      py::arg("tensor_macs_per_lane") = 0.0,
      "per-access energies from the machine's geometry and a technology node (McPAT / CACTI role)");
  m.def("ipoly_hash", &ipoly_hash);
  m.def("cache_set_index", [](const std::string& geom, uint64_t addr) {
    return cache_set_index(parse_cache_geom(geom), addr);
  });
  m.def("parse_cache", [](const std::string& geom) {
    CacheGeom g = parse_cache_geom(geom);
    py::dict d;
    d["nsets"] = g.nsets;
    d["assoc"] = g.assoc;
    d["line"] = g.line;
    d["sectored"] = g.sectored;
    d["repl"] = g.repl;
    d["wpolicy"] = g.wpolicy;
    d["alloc"] = std::string(1, (char)g.alloc);
    d["walloc"] = std::string(1, (char)g.walloc);
    d["set_index"] = g.set_index;
    d["mshr_entries"] = g.mshr_entries;
    d["mshr_merge"] = g.mshr_merge;
    d["miss_queue"] = g.miss_queue;
    d["disabled"] = g.disabled;
    return d;
  });
  m.def("decode_opcode", [](const std::string& op, uint32_t bv) {
    OpInfo o = decode_opcode(op, bv);
    py::dict d;
    d["opcode"] = o.opcode;
    d["cls"] = o.cls;
    d["space"] = o.space;
    d["flags"] = o.flags;
    d["width"] = o.width;
    d["half_ii"] = o.half_ii;
    d["known"] = o.known;
    return d;
  });
  m.def("smem_conflict_degree",
        [](const std::vector<uint64_t>& addrs, uint64_t mask, uint32_t width, const std::vector<std::string>& args) {
          SimCfg c = cfg_from_args(args);
          std::vector<uint64_t> a(64, 0);
          for (size_t i = 0; i < addrs.size() && i < 64; ++i) a[i] = addrs[i];
          return smem_conflict_degree(a.data(), mask, width, c, c.warp_size);
        });
  // CDNA4 lane-group banking of one ds_* instruction (opcode name, wave64)
  m.def("smem_conflict_degree_cdna", [](const std::vector<uint64_t>& addrs, uint64_t mask, uint32_t width,
                                        const std::string& opcode, const std::vector<std::string>& args) {
    SimCfg c = cfg_from_args(args);
    std::vector<uint64_t> a(64, 0);
    for (size_t i = 0; i < addrs.size() && i < 64; ++i) a[i] = addrs[i];
    std::string op = opcode;
    for (auto& ch : op) ch = (char)tolower(ch);
    return smem_conflict_degree(a.data(), mask, width, c, 64, lds_groups_for(op));
  });
  m.def("occupancy", [](const std::vector<std::string>& args, uint32_t threads, uint32_t shmem, uint32_t regs) {
    SimCfg c = cfg_from_args(args);
    Occupancy o = compute_occupancy(c, KernelShape{threads, shmem, regs, 1});
    py::dict d;
    d["cta_per_sm"] = o.cta_per_sm;
    d["l1_sets"] = o.l1_sets;
    d["l1_assoc"] = o.l1_assoc;
    d["shmem_kb"] = o.shmem_kb;
    d["limiter"] = std::string(o.limiter);
    return d;
  });
  m.def("parse_commandlist", [](const std::string& p) {
    py::list out;
    for (auto& c : parse_commandlist(p)) {
      py::dict d;
      d["type"] = (int)c.type;
      d["text"] = c.text;
      d["addr"] = c.addr;
      d["bytes"] = c.bytes;
      d["coll"] = c.coll;
      d["count"] = c.count;
      d["dtype_bytes"] = c.dtype_bytes;
      d["nranks"] = c.nranks;
      d["redop"] = c.redop;
      out.append(d);
    }
    return out;
  });
  m.def("kernel_info", [](const std::string& p) {
    HostKernel k = load_kernel(p);
    py::dict d;
    d["name"] = k.h.name;
    d["grid"] = std::vector<uint32_t>{k.h.grid[0], k.h.grid[1], k.h.grid[2]};
    d["block"] = std::vector<uint32_t>{k.h.block[0], k.h.block[1], k.h.block[2]};
    d["shmem"] = k.h.shmem;
    d["nregs"] = k.h.nregs;
    d["binary_version"] = k.h.binary_version;
    d["warp_insts"] = k.warp_insts;
    d["thread_insts"] = k.thread_insts;
    d["n_cta"] = k.n_cta;
    d["warps_per_cta"] = k.warps_per_cta;
    d["unknown_opcodes"] = k.unknown_opcodes;
    d["n_mems"] = (uint64_t)k.mems.size();
    return d;
  });
  m.def("convert_trace", [](const std::string& in, const std::string& out) {
    HostKernel k = load_kernel_text(in);
    if (out.size() > 6 && out.compare(out.size() - 6, 6, ".asimk") == 0)
      save_kernel_binary(k, out);
    else
      save_kernel_text(k, out);
    return k.warp_insts;
  });
  // host coalescer vs the MI355X matrix-core coalescer on one kernel: equal
  // instruction and access arrays, and where the work ran
  auto ingest_cmp = [](const HostKernel& k, const SimCfg& c, int device) {
    py::dict d;
    const auto t0 = std::chrono::steady_clock::now();
    ReadyKernel h = coalesce_kernel(k, c);
    const auto t1 = std::chrono::steady_clock::now();
    IngestStats st;
    ReadyKernel g;
    const bool ran = gpu_coalesce_kernel(k, c, device, g, &st);
    d["ran"] = ran;
    d["host_s"] = std::chrono::duration<double>(t1 - t0).count();
    d["n_insts"] = (uint64_t)h.insts.size();
    d["n_accs"] = (uint64_t)h.accs.size();
    if (!ran) return d;
    int64_t bad_inst = -1, bad_acc = -1;
    for (size_t i = 0; i < h.insts.size() && i < g.insts.size() && bad_inst < 0; ++i)
      if (memcmp(&h.insts[i], &g.insts[i], sizeof(TInst)) != 0) bad_inst = (int64_t)i;
    for (size_t i = 0; i < h.accs.size() && i < g.accs.size() && bad_acc < 0; ++i)
      if (memcmp(&h.accs[i], &g.accs[i], sizeof(TAcc)) != 0) bad_acc = (int64_t)i;
    d["equal"] = bad_inst < 0 && bad_acc < 0 && h.insts.size() == g.insts.size() && h.accs.size() == g.accs.size();
    d["first_bad_inst"] = bad_inst;
    d["first_bad_acc"] = bad_acc;
    if (bad_inst >= 0) {
      d["host_width"] = (int)h.insts[bad_inst].width;
      d["dev_width"] = (int)g.insts[bad_inst].width;
    }
    d["smem_device"] = st.smem_jobs;
    d["smem_host"] = st.smem_host;
    d["gmem_device"] = st.gmem_jobs;
    d["gmem_host"] = st.gmem_host;
    d["mfma"] = st.mfma;
    d["device_s"] = st.device_s;
    d["total_s"] = st.total_s;
    return d;
  };
  m.def("ingest_compare", [ingest_cmp](const std::string& path, const std::vector<std::string>& args, int device) {
    SimCfg c = cfg_from_args(args);
    return ingest_cmp(load_kernel(path), c, device);
  }, py::arg("path"), py::arg("args"), py::arg("device") = 0);
  // explicit instructions: (space 'shared'|'global', bytes per lane, active mask, active lanes' addresses,
  // CDNA opcode name or "")
  m.def("ingest_compare_lanes",
        [ingest_cmp](const std::vector<std::tuple<std::string, uint32_t, uint64_t, std::vector<uint64_t>, std::string>>& ins,
                     const std::vector<std::string>& args, int device) {
          SimCfg c = cfg_from_args(args);
          HostKernel k;
          k.h.name = "ingest_lanes";
          k.h.warp_size = c.warp_size ? c.warp_size : 32;
          k.n_cta = 1;
          k.warps_per_cta = 1;
          for (const auto& t : ins) {
            TInst in{};
            in.cls = OC_LOAD;
            in.space = std::get<0>(t) == "shared" ? S_SHARED : S_GLOBAL;
            in.width = (uint8_t)std::get<1>(t);
            in.mask = std::get<2>(t);
            if (!std::get<4>(t).empty()) in.opcode = decode_opcode(std::get<4>(t), 950).opcode;
            const auto& a = std::get<3>(t);
            if ((size_t)__builtin_popcountll(in.mask) != a.size()) throw std::runtime_error("one address per active lane");
            TMem m{};
            m.list = (uint32_t)k.addrs.size();
            k.addrs.insert(k.addrs.end(), a.begin(), a.end());
            in.mem = (uint32_t)k.mems.size();
            k.mems.push_back(m);
            k.insts.push_back(in);
          }
          k.streams.push_back(WStream{0, (uint32_t)k.insts.size()});
          return ingest_cmp(k, c, device);
        },
        py::arg("insts"), py::arg("args"), py::arg("device") = 0);
  // host streaming: the per-CTA reader's instructions, accesses and warp
  // streams equal the whole-kernel load's, window by window (CTAs [lo, lo+step)
  // resident, the ones below dropped)
  m.def("stream_compare", [](const std::string& path, const std::vector<std::string>& args, uint32_t step) {
    SimCfg c = cfg_from_args(args);
    ReadyKernel w = coalesce_kernel(load_kernel_text(path), c);
    ReadyKernel r = open_streamed_kernel(path, c);
    const uint32_t wpc = w.warps_per_cta;
    int64_t bad_cta = -1;
    step = std::max<uint32_t>(1, step);
    for (uint32_t lo = 0; lo < w.n_cta && bad_cta < 0; lo += step) {
      const uint32_t hi = std::min(w.n_cta, lo + step);
      r.resident(lo, hi);
      for (uint32_t cta = lo; cta < hi && bad_cta < 0; ++cta)
        for (uint32_t wi = 0; wi < wpc && bad_cta < 0; ++wi) {
          const WStream& a = w.streams[(size_t)cta * wpc + wi];
          const WStream& b = r.streams[(size_t)(cta - r.cta_lo) * wpc + wi];
          if (a.count != b.count) bad_cta = cta;
          for (uint32_t j = 0; j < a.count && bad_cta < 0; ++j) {
            TInst x = w.insts[a.begin + j];
            TInst y = r.insts[((b.begin + j) - (r.ibase & kStreamInstMask)) & kStreamInstMask];
            const uint32_t xm = x.mem, ym = y.mem;
            x.mem = y.mem = 0;
            if (memcmp(&x, &y, sizeof(TInst)) != 0 || (xm == kNoMem) != (ym == kNoMem)) {
              bad_cta = cta;
              break;
            }
            if (xm == kNoMem) continue;
            const uint64_t yl = (ym - (r.abase & kStreamAccMask)) & kStreamAccMask;
            for (uint32_t q = 0; q < x.width && bad_cta < 0; ++q)
              if (memcmp(&w.accs[xm + q], &r.accs[yl + q], sizeof(TAcc)) != 0) bad_cta = cta;
          }
        }
    }
    py::dict d;
    d["equal"] = bad_cta < 0;
    d["bad_cta"] = bad_cta;
    d["whole_bytes"] = w.host_bytes();
    d["stream_peak_bytes"] = r.host_peak_bytes;
    d["n_cta"] = w.n_cta;
    return d;
  });
  m.def("coalesce_summary", [](const std::string& path, const std::vector<std::string>& args) {
    SimCfg c = cfg_from_args(args);
    ReadyKernel r = coalesce_kernel(load_kernel(path), c);
    py::dict d;
    d["n_accs"] = (uint64_t)r.accs.size();
    uint64_t mem = 0, shared_deg = 0, nshared = 0;
    for (auto& in : r.insts) {
      if (in.mem != kNoMem) mem++;
      if ((in.cls == OC_LOAD || in.cls == OC_STORE) && in.space == S_SHARED) {
        nshared++;
        shared_deg += in.width;
      }
    }
    d["mem_insts"] = mem;
    d["shared_insts"] = nshared;
    d["shared_degree_sum"] = shared_deg;
    py::list acc;
    for (size_t i = 0; i < r.accs.size() && i < 4096; ++i)
      acc.append(py::make_tuple(r.accs[i].line, r.accs[i].sectors, r.accs[i].bytes));
    d["accs"] = acc;
    return d;
  });

  py::class_<Simulator>(m, "Simulator")
      .def(py::init([](const std::vector<std::string>& args, bool echo) {
             // construction parses the configuration and builds the engine
             // (the GPU engine allocates and uploads every unit's state):
             // without the GIL, so the node bench's worker threads set up
             // their simulations concurrently
             py::gil_scoped_release nogil;
             auto* s = new Simulator(args);
             s->set_echo(echo);
             return s;
           }),
           py::arg("args"), py::arg("echo") = false)
      .def("run", &Simulator::run, py::call_guard<py::gil_scoped_release>())
      .def("run_command", &Simulator::run_command, py::call_guard<py::gil_scoped_release>())
      .def("num_commands", [](Simulator& s) { return s.commands().size(); })
      .def("load_commands", &Simulator::load_commands, py::call_guard<py::gil_scoped_release>())
      .def("print_header", [](Simulator& s) { s.load_commands(); })
      .def_property_readonly("output", &Simulator::output)
      .def_property_readonly("tot_cycle", &Simulator::tot_cycle)
      .def_property_readonly("tot_insn", &Simulator::tot_insn)
      .def_property_readonly("sim_seconds", &Simulator::sim_seconds)
      .def_property_readonly("wall_seconds", &Simulator::wall_seconds)
      .def_property_readonly("deadlock", &Simulator::deadlock)
      .def_property_readonly("engine", [](Simulator& s) { return std::string(s.engine().name()); })
      .def_property_readonly("config", [](Simulator& s) { return cfg_dict(s.cfg()); })
      .def_property_readonly("kernels",
                             [](Simulator& s) {
                               py::list l;
                               for (auto& k : s.kernels()) l.append(kernel_dict(k));
                               return l;
                             })
      .def_property_readonly("collectives",
                             [](Simulator& s) {
                               py::list l;
                               for (auto& c : s.collectives()) {
                                 py::dict d;
                                 d["op"] = c.op;
                                 d["bytes"] = c.bytes;
                                 d["nranks"] = c.nranks;
                                 d["cycles"] = c.cycles;
                                 l.append(d);
                               }
                               return l;
                             })
      .def("collective_cycles",
           [](Simulator& s, const std::string& line) { return s.collective_cycles(parse_collective_line(line)); })
      .def("link_params", [](Simulator& s) { return link_dict(s.link_params()); })
      .def("dump_pipeline", &Simulator::dump_pipeline, py::arg("sm") = -1, py::arg("channel") = -1,
           "pipeline state of an SM / memory channel (-1: all busy SMs / all channels, -2: none)")
      .def_property_readonly("core_period_ps", &Simulator::core_period_ps)
      .def("set_collective_hook",
           [](Simulator& s, py::function f) {
             s.set_collective_hook([f](const Command& c, uint64_t now) -> uint64_t {
               py::gil_scoped_acquire g;
               py::dict d;
               d["op"] = c.coll;
               d["bytes"] = c.bytes;
               d["count"] = c.count;
               d["dtype_bytes"] = c.dtype_bytes;
               d["nranks"] = c.nranks;
               d["root"] = c.root;
               d["text"] = c.text;
               return f(d, now).cast<uint64_t>();
             });
           })
      .def("snapshot",
           [](Simulator& s) {
             std::vector<uint8_t> v;
             s.engine().snapshot(v);
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
           })
      .def("restore", [](Simulator& s, py::bytes b) {
        std::string str = b;
        std::vector<uint8_t> v(str.begin(), str.end());
        s.engine().restore(v);
      });

  py::class_<LinkSim>(m, "LinkSim")
      .def(py::init([](const py::dict& p, const std::string& kind, uint64_t bytes, int root, int rank, int world,
                       uint64_t start_ps) { return new LinkSim(link_from(p), coll_from(kind, bytes, root), rank, world,
                                                              start_ps); }),
           py::arg("params"), py::arg("kind"), py::arg("bytes"), py::arg("root"), py::arg("rank"), py::arg("world"),
           py::arg("start_ps"))
      .def("emit",
           [](LinkSim& l, uint64_t t_end) {
             std::vector<LinkPkt> out;
             l.emit(t_end, out);
             return py::bytes(reinterpret_cast<const char*>(out.data()), out.size() * sizeof(LinkPkt));
           })
      .def("receive",
           [](LinkSim& l, py::bytes b) {
             std::string s = b;
             if (s.size() % sizeof(LinkPkt)) throw std::invalid_argument("LinkSim.receive: ragged packet buffer");
             std::vector<LinkPkt> v(s.size() / sizeof(LinkPkt));
             if (!v.empty()) memcpy(v.data(), s.data(), s.size());
             l.receive(v.data(), v.size());
           })
      .def("next_event", &LinkSim::next_event)
      .def("done", &LinkSim::done)
      .def_property_readonly("finish_ps", &LinkSim::finish_ps)
      .def_property_readonly("epoch_ps", &LinkSim::epoch_ps)
      .def_property_readonly("channels", &LinkSim::channels)
      .def_property_readonly("packets_sent", &LinkSim::packets_sent)
      .def_readonly_static("packet_bytes", &kLinkPktBytes)
      // one epoch of the packet exchange, packed into / unpacked from the
      // all-to-all buffers in place (parallel/collectives.py)
      .def("pack_epoch",
           [](LinkSim& l, uint64_t t_end, int k, int hdr, int64_t ann_next, int64_t ann_busy,
              py::array_t<int64_t, py::array::c_style> send) {
             const size_t need = (size_t)l.world() * ((size_t)hdr + 4 * (size_t)k);
             if ((size_t)send.size() != need) throw std::invalid_argument("pack_epoch: send buffer size");
             EpochOut o;
             pack_epoch(l, t_end, k, hdr, ann_next, ann_busy, send.mutable_data(), o);
             py::array_t<int64_t> extra(o.extra.size());
             if (!o.extra.empty()) memcpy(extra.mutable_data(), o.extra.data(), o.extra.size() * sizeof(int64_t));
             return py::make_tuple(extra, o.extra_words, o.packets, o.max_count);
           })
      .def("unpack_epoch",
           [](LinkSim& l, py::array_t<int64_t, py::array::c_style | py::array::forcecast> recv, int k, int hdr,
              py::array_t<int64_t, py::array::c_style | py::array::forcecast> extra) {
             const size_t need = (size_t)l.world() * ((size_t)hdr + 4 * (size_t)k);
             if ((size_t)recv.size() != need) throw std::invalid_argument("unpack_epoch: recv buffer size");
             EpochIn r = unpack_epoch(l, recv.data(), k, hdr, extra.size() ? extra.data() : nullptr, (size_t)extra.size());
             return py::make_tuple(r.any_busy, r.next);
           });

  m.def(
      "linksim_run_local",
      [](const py::dict& p, const std::string& kind, uint64_t bytes, int root, const std::vector<uint64_t>& start) {
        uint64_t ep = 0, pk = 0;
        auto fin = linksim_run_local(link_from(p), coll_from(kind, bytes, root), start, &ep, &pk);
        py::dict d;
        d["finish_ps"] = fin;
        d["epochs"] = ep;
        d["packets"] = pk;
        return d;
      },
      py::arg("params"), py::arg("kind"), py::arg("bytes"), py::arg("root"), py::arg("start_ps"));

  py::class_<PowerModel>(m, "PowerModel")
      .def(py::init<>())
      .def("load_xml",
           [](PowerModel& p, const std::string& path) {
             std::string err;
             if (!p.load_xml(path, &err)) throw std::runtime_error(err);
           })
      .def("set_param", &PowerModel::set_param)
      .def("param", &PowerModel::param, py::arg("name"), py::arg("default") = 0.0)
      .def("coefficients", &PowerModel::coefficients)
      .def_static("activity_names",
                  []() {
                    std::vector<std::string> v;
                    for (int i = 0; i < PA_COUNT; ++i) v.push_back(kPwrActName[i]);
                    return v;
                  })
      .def_static("base_nj", &PowerModel::base_nj)
      .def("compute_hw",
           [](PowerModel& p, const std::string& csv, const std::string& bench, const std::string& kernel,
              double mhz, uint32_t n_sm) {
             Activity a;
             if (!PowerModel::activity_from_hw_csv(csv, bench, kernel, a, n_sm)) throw std::runtime_error("row not found");
             PowerReport r = p.compute(a, mhz, n_sm);
             py::dict d;
             d["total"] = r.total;
             d["dynamic"] = r.dynamic;
             d["static"] = r.static_w;
             d["constant"] = r.constant;
             d["idle"] = r.idle;
             d["category"] = r.static_category;
             std::vector<double> act(a.a, a.a + PA_COUNT);
             d["activity"] = act;
             d["cycles"] = a.cycles;
             d["idle_sms"] = a.idle_sms;
             return d;
           });
}
