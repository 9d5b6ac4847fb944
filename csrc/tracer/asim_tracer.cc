// rocprofiler-sdk tool: API-level trace capture on MI355X.
//
// Counterpart of the host side of the reference's NVBit tracer
// (util/tracer_nvbit/tracer_tool/tracer_tool.cu: nvbit_at_cuda_event for
// memcpy :369-378 and kernel launches :380-506, and the NCCL interposers
// :800-859 that append the collective's *name* to kernelslist).  Loaded with
//   ROCP_TOOL_LIBRARIES=bin/libasim_tracer.so ASIM_TRACE_DIR=<dir> <app>
// it records, per process:
//  * every RCCL collective / group / communicator call with its arguments
//    (count, datatype, reduction op, root, communicator size and rank) as a
//    kernelslist.g line -- the reference drops the arguments;
//  * every kernel dispatch (name, grid, workgroup, LDS, VGPR/AGPR/SGPR counts,
//    scratch) in dispatches.csv, and -- with ASIM_TRACE_TOOL_LIST=1, for
//    applications without asim_trace annotations -- header-only
//    kernel-N.traceg files plus MemcpyHtoD lines in kernelslist.g;
//  * kernel-range filtering (ASIM_TRACE_KERNEL_START/END) and a device filter
//    (ASIM_TRACE_GPU = agent node id).
#include <filesystem>
#include <dlfcn.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

namespace {

struct KSym {
  std::string name;
  uint32_t lds = 0, scratch = 0, sgpr = 0, vgpr = 0, agpr = 0;
};

struct Tool {
  std::string dir = ".";
  bool full_list = false;
  long kstart = 0, kend = 1L << 40;
  std::mutex mu;
  std::unordered_map<uint64_t, KSym> syms;
  std::atomic<long> dispatches{0};
  rocprofiler_context_id_t ctx{0};

  void line(const std::string& file, const std::string& s) {
    std::lock_guard<std::mutex> g(mu);
    FILE* f = fopen((dir + "/" + file).c_str(), "a");
    if (!f) return;
    fprintf(f, "%s\n", s.c_str());
    fclose(f);
  }
};

Tool* g_tool = nullptr;

const char* nccl_dtype(int t) {
  static const char* n[] = {"ncclInt8",    "ncclUint8",   "ncclInt32",   "ncclUint32",  "ncclInt64",
                            "ncclUint64",  "ncclFloat16", "ncclFloat32", "ncclFloat64", "ncclBfloat16"};
  return t >= 0 && t < 10 ? n[t] : "ncclFloat32";
}

const char* nccl_op(int o) {
  static const char* n[] = {"ncclSum", "ncclProd", "ncclMax", "ncclMin", "ncclAvg"};
  return o >= 0 && o < 5 ? n[o] : "ncclSum";
}

// size / rank of a communicator through the application's own librccl
void comm_info(void* comm, int* nranks, int* rank) {
  using F = int (*)(void*, int*);
  static F count = (F)dlsym(RTLD_DEFAULT, "ncclCommCount");
  static F user_rank = (F)dlsym(RTLD_DEFAULT, "ncclCommUserRank");
  *nranks = 1;
  *rank = 0;
  if (comm && count) count(comm, nranks);
  if (comm && user_rank) user_rank(comm, rank);
}

void rccl_cb(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.phase != ROCPROFILER_CALLBACK_PHASE_ENTER) return;
  auto* d = static_cast<rocprofiler_callback_tracing_rccl_api_data_t*>(rec.payload);
  const auto& a = d->args;
  char buf[512];
  int n = 1, r = 0;
  switch (rec.operation) {
    case ROCPROFILER_RCCL_API_ID_ncclAllReduce:
      comm_info(a.ncclAllReduce.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclAllReduce,count=%zu,dtype=%s,op=%s,nranks=%d,rank=%d", a.ncclAllReduce.count,
               nccl_dtype((int)a.ncclAllReduce.datatype), nccl_op((int)a.ncclAllReduce.op), n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclAllGather:
      comm_info(a.ncclAllGather.comm, &n, &r);
      // total buffer = sendcount * nranks (the analytic/packet models take the full size)
      snprintf(buf, sizeof(buf), "ncclAllGather,count=%zu,dtype=%s,nranks=%d,rank=%d",
               a.ncclAllGather.sendcount * (size_t)n, nccl_dtype((int)a.ncclAllGather.datatype), n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclReduceScatter:
      comm_info(a.ncclReduceScatter.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclReduceScatter,count=%zu,dtype=%s,op=%s,nranks=%d,rank=%d",
               a.ncclReduceScatter.recvcount * (size_t)n, nccl_dtype((int)a.ncclReduceScatter.datatype),
               nccl_op((int)a.ncclReduceScatter.op), n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclBroadcast:
      comm_info(a.ncclBroadcast.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclBroadcast,count=%zu,dtype=%s,root=%d,nranks=%d,rank=%d", a.ncclBroadcast.count,
               nccl_dtype((int)a.ncclBroadcast.datatype), a.ncclBroadcast.root, n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclReduce:
      comm_info(a.ncclReduce.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclReduce,count=%zu,dtype=%s,op=%s,root=%d,nranks=%d,rank=%d", a.ncclReduce.count,
               nccl_dtype((int)a.ncclReduce.datatype), nccl_op((int)a.ncclReduce.op), a.ncclReduce.root, n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclAllToAll:
      comm_info(a.ncclAllToAll.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclAllToAll,count=%zu,dtype=%s,nranks=%d,rank=%d",
               a.ncclAllToAll.count * (size_t)n, nccl_dtype((int)a.ncclAllToAll.datatype), n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclSend:
      comm_info(a.ncclSend.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclSend,count=%zu,dtype=%s,peer=%d,nranks=%d,rank=%d", a.ncclSend.count,
               nccl_dtype((int)a.ncclSend.datatype), a.ncclSend.peer, n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclRecv:
      comm_info(a.ncclRecv.comm, &n, &r);
      snprintf(buf, sizeof(buf), "ncclRecv,count=%zu,dtype=%s,peer=%d,nranks=%d,rank=%d", a.ncclRecv.count,
               nccl_dtype((int)a.ncclRecv.datatype), a.ncclRecv.peer, n, r);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclGroupStart: snprintf(buf, sizeof(buf), "ncclGroupStart"); break;
    case ROCPROFILER_RCCL_API_ID_ncclGroupEnd: snprintf(buf, sizeof(buf), "ncclGroupEnd"); break;
    case ROCPROFILER_RCCL_API_ID_ncclCommInitAll:
      snprintf(buf, sizeof(buf), "ncclCommInitAll,nranks=%d", a.ncclCommInitAll.ndev);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclCommInitRank:
      snprintf(buf, sizeof(buf), "ncclCommInitRank,nranks=%d,rank=%d", a.ncclCommInitRank.nranks,
               a.ncclCommInitRank.myrank);
      break;
    case ROCPROFILER_RCCL_API_ID_ncclCommDestroy: snprintf(buf, sizeof(buf), "ncclCommDestroy"); break;
    default: return;
  }
  g_tool->line("kernelslist.g", buf);
}

void code_object_cb(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.operation != ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER) return;
  if (rec.phase != ROCPROFILER_CALLBACK_PHASE_LOAD) return;
  auto* d = static_cast<rocprofiler_callback_tracing_code_object_kernel_symbol_register_data_t*>(rec.payload);
  KSym s;
  s.name = d->kernel_name ? d->kernel_name : "unknown";
  if (s.name.size() > 3 && s.name.compare(s.name.size() - 3, 3, ".kd") == 0) s.name.resize(s.name.size() - 3);
  s.lds = d->group_segment_size;
  s.scratch = d->private_segment_size;
  s.sgpr = d->sgpr_count;
  s.vgpr = d->arch_vgpr_count;
  s.agpr = d->accum_vgpr_count;
  std::lock_guard<std::mutex> g(g_tool->mu);
  g_tool->syms[d->kernel_id] = s;
}

void dispatch_cb(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.operation != ROCPROFILER_KERNEL_DISPATCH_ENQUEUE || rec.phase != ROCPROFILER_CALLBACK_PHASE_ENTER) return;
  auto* d = static_cast<rocprofiler_callback_tracing_kernel_dispatch_data_t*>(rec.payload);
  const auto& di = d->dispatch_info;
  const long id = ++g_tool->dispatches;
  if (id < g_tool->kstart || id > g_tool->kend) return;
  KSym s;
  {
    std::lock_guard<std::mutex> g(g_tool->mu);
    auto it = g_tool->syms.find(di.kernel_id);
    if (it != g_tool->syms.end()) s = it->second;
  }
  // grid_size is in work-items (HSA); the trace format wants workgroups
  const uint32_t wx = di.workgroup_size.x ? di.workgroup_size.x : 1, wy = di.workgroup_size.y ? di.workgroup_size.y : 1,
                 wz = di.workgroup_size.z ? di.workgroup_size.z : 1;
  const uint32_t gx = (di.grid_size.x + wx - 1) / wx, gy = (di.grid_size.y + wy - 1) / wy,
                 gz = (di.grid_size.z + wz - 1) / wz;
  char buf[1024];
  snprintf(buf, sizeof(buf), "%ld,%s,%u,%u,%u,%u,%u,%u,%u,%u,%u,%u,%u,%llu", id, s.name.c_str(), gx, gy, gz, wx, wy,
           wz, di.group_segment_size, di.private_segment_size, s.vgpr, s.agpr, s.sgpr,
           (unsigned long long)di.dispatch_id);
  g_tool->line("dispatches.csv", buf);
  if (!g_tool->full_list) return;
  const std::string fn = "kernel-" + std::to_string(id) + ".traceg";
  FILE* f = fopen((g_tool->dir + "/" + fn).c_str(), "w");
  if (f) {
    fprintf(f, "-kernel name = %s\n-kernel id = %ld\n-grid dim = (%u,%u,%u)\n-block dim = (%u,%u,%u)\n", s.name.c_str(),
            id, gx, gy, gz, wx, wy, wz);
    fprintf(f, "-shmem = %u\n-nregs = %u\n-binary version = 950\n-wavefront size = 64\n-hip stream id = 0\n",
            di.group_segment_size, s.vgpr + s.agpr);
    fprintf(f, "-rocprofiler version = asim_tracer\n-accelsim tracer version = 4\n\n");
    fprintf(f, "#traces format = PC mask dest_num reg_dests opcode src_num reg_srcs mem_width mem_addresses\n");
    fprintf(f, "# header only: instruction records come from asim_trace-annotated builds\n");
    fclose(f);
  }
  g_tool->line("kernelslist.g", fn);
}

void memcpy_cb(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (!g_tool->full_list || rec.phase != ROCPROFILER_CALLBACK_PHASE_EXIT) return;
  if (rec.operation != ROCPROFILER_MEMORY_COPY_HOST_TO_DEVICE) return;
  auto* d = static_cast<rocprofiler_callback_tracing_memory_copy_data_t*>(rec.payload);
  char buf[128];
  snprintf(buf, sizeof(buf), "MemcpyHtoD,0x%016llx,%llu", (unsigned long long)d->dst_address.value,
           (unsigned long long)d->bytes);
  g_tool->line("kernelslist.g", buf);
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  auto ok = [](rocprofiler_status_t s) { return s == ROCPROFILER_STATUS_SUCCESS; };
  if (!ok(rocprofiler_create_context(&g_tool->ctx))) return -1;
  rocprofiler_configure_callback_tracing_service(g_tool->ctx, ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT, nullptr, 0,
                                                 code_object_cb, nullptr);
  rocprofiler_configure_callback_tracing_service(g_tool->ctx, ROCPROFILER_CALLBACK_TRACING_KERNEL_DISPATCH, nullptr,
                                                 0, dispatch_cb, nullptr);
  rocprofiler_configure_callback_tracing_service(g_tool->ctx, ROCPROFILER_CALLBACK_TRACING_MEMORY_COPY, nullptr, 0,
                                                 memcpy_cb, nullptr);
  rocprofiler_configure_callback_tracing_service(g_tool->ctx, ROCPROFILER_CALLBACK_TRACING_RCCL_API, nullptr, 0,
                                                 rccl_cb, nullptr);
  return ok(rocprofiler_start_context(g_tool->ctx)) ? 0 : -1;
}

void tool_fini(void*) {
  if (g_tool) g_tool->line("dispatches.csv.done", std::to_string(g_tool->dispatches.load()));
}

}  // namespace

extern "C" rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                                      rocprofiler_client_id_t* id) {
  id->name = "asim_tracer";
  g_tool = new Tool();
  if (const char* d = getenv("ASIM_TRACE_DIR")) g_tool->dir = d;
  if (const char* s = getenv("ASIM_TRACE_TOOL_LIST")) g_tool->full_list = atoi(s) != 0;
  if (const char* s = getenv("ASIM_TRACE_KERNEL_START")) g_tool->kstart = atol(s);
  if (const char* s = getenv("ASIM_TRACE_KERNEL_END")) g_tool->kend = atol(s);
  {
    std::error_code ec;
    std::filesystem::create_directories(g_tool->dir, ec);
    if (ec) fprintf(stderr, "asim_tracer: cannot create %s\n", g_tool->dir.c_str());
  }
  g_tool->line("dispatches.csv", "id,kernel,grid_x,grid_y,grid_z,wg_x,wg_y,wg_z,lds,scratch,vgpr,agpr,sgpr,dispatch_id");
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini,
                                                 nullptr};
  return &cfg;
}
