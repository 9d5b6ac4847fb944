// L1 associativity and set count (reference GPU_Microbenchmark
// l1_cache/l1_assoc): one lane pointer-chases N lines placed `span` bytes
// apart.  With span = sets x line size every line maps to one set, so the
// chain stays an L1 hit up to N = associativity and turns into an L2 hit
// beyond; the smallest span that shows the knee gives the set count.
// Prints the measured geometry and the -gpgpu_cache:dl1 line.
#include "ubench.h"

int main() {
  UbDevice d;
  const int iters = 4096, line = 128;
  const double l1 = ub_chase_latency(8 * 1024, line, iters);  // all-hit reference
  printf("# l1_hit_latency %.1f\n", l1);
  int assoc = 0, sets = 0;
  for (size_t span = 1024; span <= 64 * 1024 && !assoc; span *= 2) {
    int knee = 0;
    for (int n = 2; n <= 32; ++n) {
      const double lat = ub_chase_latency((size_t)n * span, span, iters);
      printf("span %6zu B  lines %2d : %7.1f cycles/load\n", span, n, lat);
      if (lat > 1.3 * l1) {
        knee = n - 1;
        break;
      }
    }
    // the knee at this span: below it the lines fit the ways of one set
    if (knee > 0 && knee < 32 && (size_t)knee * span <= 64 * 1024) {
      assoc = knee;
      sets = (int)(span / line);
    }
  }
  if (assoc) {
    printf("# l1_assoc %d\n# l1_sets %d\n# l1_bytes %d\n", assoc, sets, assoc * sets * line);
    char v[128];
    snprintf(v, sizeof(v), "S:%d:%d:%d,L:T:m:L:L,A:256:8,16:0,32", sets, line, assoc);
    ub_opt("-gpgpu_cache:dl1", v);
  } else {
    printf("# l1 associativity not resolved (hashed set index?)\n");
  }
  return 0;
}
