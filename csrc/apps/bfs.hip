// bfs-shaped breadth-first search (Rodinia bfs: frontier mask kernel that
// scans each frontier node's edge list, then an update kernel; the host loops
// while any node changed), plain HIP.  Irregular, data-dependent accesses and
// divergence.
#include <cmath>

#include "app_common.h"

__global__ void Kernel(const int2* nodes, const int* edges, int* mask, const int* visited, int* updating, int* cost,
                       int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && mask[i]) {
    mask[i] = 0;
    const int2 nd = nodes[i];
    const int c = cost[i];
    for (int e = nd.x; e < nd.x + nd.y; ++e) {
      const int id = edges[e];
      if (!visited[id]) {
        cost[id] = c + 1;
        updating[id] = 1;
      }
    }
  }
}

__global__ void Kernel2(int* mask, int* updating, int* visited, int* over, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && updating[i]) {
    mask[i] = 1;
    visited[i] = 1;
    *over = 1;
    updating[i] = 0;
  }
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
  APP_HIP(hipMalloc(&dn, n * sizeof(int2)));
  APP_HIP(hipMalloc(&de, edges.size() * 4));
  APP_HIP(hipMalloc(&dm, n * 4));
  APP_HIP(hipMalloc(&dv, n * 4));
  APP_HIP(hipMalloc(&du, n * 4));
  APP_HIP(hipMalloc(&dc, n * 4));
  APP_HIP(hipMalloc(&dover, 4));
  APP_HIP(hipMemcpy(dn, nodes.data(), n * sizeof(int2), hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(de, edges.data(), edges.size() * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(dm, mask.data(), n * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(dv, visited.data(), n * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(du, upd.data(), n * 4, hipMemcpyHostToDevice));
  APP_HIP(hipMemcpy(dc, cost.data(), n * 4, hipMemcpyHostToDevice));
  const int blk = 256, grid = (n + blk - 1) / blk;
  int over = 1, levels = 0;
  while (over && levels < 64) {
    over = 0;
    APP_HIP(hipMemcpy(dover, &over, 4, hipMemcpyHostToDevice));
    Kernel<<<grid, blk>>>(dn, de, dm, dv, du, dc, n);
    Kernel2<<<grid, blk>>>(dm, du, dv, dover, n);
    APP_HIP(hipGetLastError());
    APP_HIP(hipMemcpy(&over, dover, 4, hipMemcpyDeviceToHost));
    ++levels;
  }
  APP_HIP(hipMemcpy(cost.data(), dc, n * 4, hipMemcpyDeviceToHost));
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
  for (void* p : {(void*)dn, (void*)de, (void*)dm, (void*)dv, (void*)du, (void*)dc, (void*)dover}) APP_HIP(hipFree(p));
  return ok ? 0 : 1;
}
