// bfs-shaped breadth-first search (Rodinia bfs: frontier mask kernel that
// scans each frontier node's edge list, then an update kernel; the host loops
// while any node changed), HIP + asim_trace annotations.  Irregular,
// data-dependent accesses and divergence.
#include <cmath>

#include "../tracer/asim_trace.h"

using namespace asim_trace;

template <class TR>
__global__ void bfs_k1(TR tr, const int2* nodes, const int* edges, int* mask, const int* visited, int* updating,
                       int* cost, int n) {
  auto w = tr.wave();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  ASIM_VALU(w, V_MAD_U32_U24, 1, 0);
  ASIM_VALU(w, V_CMP_GT_I32, 0, 1);
  if (i < n) {
    const int m = ASIM_LD(w, GLOBAL_LOAD_DWORD, mask + i, 2, 1);
    ASIM_VALU(w, S_WAITCNT, 0, 0);
    ASIM_VALU(w, V_CMP_GT_I32, 0, 2);
    if (m) {
      ASIM_ST(w, GLOBAL_STORE_DWORD, mask + i, 0, 0, 1);
      const int2 nd = ASIM_LD(w, GLOBAL_LOAD_DWORDX2, nodes + i, 3, 1);
      const int c = ASIM_LD(w, GLOBAL_LOAD_DWORD, cost + i, 4, 1);
      ASIM_VALU(w, S_WAITCNT, 0, 0);
      for (int e = nd.x; e < nd.x + nd.y; ++e) {
        ASIM_VALU(w, V_ADD_U32, 5, 3);
        const int id = ASIM_LD(w, GLOBAL_LOAD_DWORD, edges + e, 6, 5);
        ASIM_VALU(w, S_WAITCNT, 0, 0);
        const int v = ASIM_LD(w, GLOBAL_LOAD_DWORD, visited + id, 7, 6);
        ASIM_VALU(w, S_WAITCNT, 0, 0);
        ASIM_VALU(w, V_CMP_GT_I32, 0, 7);
        if (!v) {
          ASIM_VALU(w, V_ADD_U32, 8, 4);
          ASIM_ST(w, GLOBAL_STORE_DWORD, cost + id, c + 1, 8, 6);
          ASIM_ST(w, GLOBAL_STORE_DWORD, updating + id, 1, 0, 6);
        }
        ASIM_VALU(w, S_CBRANCH_SCC1, 0, 0);
      }
    }
  }
  w.exit();
}

template <class TR>
__global__ void bfs_k2(TR tr, int* mask, int* updating, int* visited, int* over, int n) {
  auto w = tr.wave();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  ASIM_VALU(w, V_MAD_U32_U24, 1, 0);
  ASIM_VALU(w, V_CMP_GT_I32, 0, 1);
  if (i < n) {
    const int u = ASIM_LD(w, GLOBAL_LOAD_DWORD, updating + i, 2, 1);
    ASIM_VALU(w, S_WAITCNT, 0, 0);
    ASIM_VALU(w, V_CMP_GT_I32, 0, 2);
    if (u) {
      ASIM_ST(w, GLOBAL_STORE_DWORD, mask + i, 1, 0, 1);
      ASIM_ST(w, GLOBAL_STORE_DWORD, visited + i, 1, 0, 1);
      ASIM_ST(w, GLOBAL_STORE_DWORD, over, 1, 0, 0);
      ASIM_ST(w, GLOBAL_STORE_DWORD, updating + i, 0, 0, 1);
    }
  }
  w.exit();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 65536, deg = 6;
  std::vector<int2> nodes(n);
  std::vector<int> edges;
  uint32_t s = 7;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const int d = 1 + (int)((s >> 20) % (2 * deg - 1));
    nodes[i] = make_int2((int)edges.size(), d);
    for (int k = 0; k < d; ++k) {
      s = s * 1664525u + 1013904223u;
      // mostly-local edges plus some long jumps
      const int j = (k & 1) ? (int)((s >> 8) % n) : (i + 1 + (int)((s >> 24) % 64)) % n;
      edges.push_back(j);
    }
  }
  std::vector<int> mask(n, 0), visited(n, 0), cost(n, -1), upd(n, 0);
  mask[0] = visited[0] = 1;
  cost[0] = 0;
  int2* dn;
  int *de, *dm, *dv, *du, *dc, *dover;
  ASIM_HIP(hipMalloc(&dn, n * sizeof(int2)));
  ASIM_HIP(hipMalloc(&de, edges.size() * 4));
  ASIM_HIP(hipMalloc(&dm, n * 4));
  ASIM_HIP(hipMalloc(&dv, n * 4));
  ASIM_HIP(hipMalloc(&du, n * 4));
  ASIM_HIP(hipMalloc(&dc, n * 4));
  ASIM_HIP(hipMalloc(&dover, 4));
  memcpy_htod(dn, nodes.data(), n * sizeof(int2));
  memcpy_htod(de, edges.data(), edges.size() * 4);
  memcpy_htod(dm, mask.data(), n * 4);
  memcpy_htod(dv, visited.data(), n * 4);
  memcpy_htod(du, upd.data(), n * 4);
  memcpy_htod(dc, cost.data(), n * 4);
  const int blk = 256, grid = (n + blk - 1) / blk;
  int over = 1, levels = 0;
  while (over && levels < 64) {
    over = 0;
    ASIM_HIP(hipMemcpy(dover, &over, 4, hipMemcpyHostToDevice));
    launch("_Z6KernelP4NodePiPbS2_S2_S1_i", bfs_k1<On>, bfs_k1<Off>, dim3(grid), dim3(blk), 0, 0,
           (const int2*)dn, (const int*)de, dm, (const int*)dv, du, dc, n);
    launch("_Z7Kernel2PbS_S_S_i", bfs_k2<On>, bfs_k2<Off>, dim3(grid), dim3(blk), 0, 0, dm, du, dv, dover, n);
    ASIM_HIP(hipMemcpy(&over, dover, 4, hipMemcpyDeviceToHost));
    ++levels;
  }
  ASIM_HIP(hipMemcpy(cost.data(), dc, n * 4, hipMemcpyDeviceToHost));
  // host BFS check
  std::vector<int> ref(n, -1), q{0};
  ref[0] = 0;
  for (size_t h = 0; h < q.size(); ++h)
    for (int e = nodes[q[h]].x; e < nodes[q[h]].x + nodes[q[h]].y; ++e)
      if (ref[edges[e]] < 0) {
        ref[edges[e]] = ref[q[h]] + 1;
        q.push_back(edges[e]);
      }
  const bool ok = ref == cost;
  printf("bfs n=%d levels=%d: %s\n", n, levels, ok ? "PASSED" : "FAILED");
  for (void* p : {(void*)dn, (void*)de, (void*)dm, (void*)dv, (void*)du, (void*)dc, (void*)dover}) ASIM_HIP(hipFree(p));
  return ok ? 0 : 1;
}
