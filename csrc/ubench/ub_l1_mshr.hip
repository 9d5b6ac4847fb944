// Outstanding-miss capacity of the vector L1 (reference GPU_Microbenchmark
// l1_cache/l1_mshr): one wavefront issues N independent loads, each to its own
// never-touched 128-byte line (so every load misses L1 and L2 and goes to
// HBM), then waits for all of them.  While N fits the L1's miss-handling
// capacity the time is one memory latency plus N issue slots; past it the
// wave needs a second round trip, and the time per batch steps up.  The knee
// is the number of misses one CU keeps in flight for one wave.
#include "ubench.h"

template <int N>
__global__ void ub_mshr_kernel(const float* __restrict__ base, size_t region, int reps, uint64_t* out) {
  float acc = 0.f;
  uint64_t total = 0;
  for (int r = 0; r < reps; ++r) {
    const float* p = base + (size_t)r * region / sizeof(float);
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t0 = ub_clock();
    float v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = __builtin_nontemporal_load(p + (size_t)i * 4096 + threadIdx.x);
#pragma unroll
    for (int i = 0; i < N; ++i) acc += v[i];
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = ub_clock();
    total += t1 - t0;
  }
  if (threadIdx.x == 0) {
    out[0] = total / (uint64_t)reps;
    out[1] = (uint64_t)acc;
  }
}

template <int N>
double run(float* buf, size_t region, int reps, uint64_t* o) {
  hipLaunchKernelGGL(ub_mshr_kernel<N>, dim3(1), dim3(32), 0, 0, buf, region, reps, o);
  UB_CHECK(hipDeviceSynchronize());
  uint64_t r[2];
  UB_CHECK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
  return (double)r[0];
}

int main() {
  UbDevice d;
  // every (batch, load) pair gets its own 16 KB-apart line: nothing is reused
  const int reps = 24;
  const size_t region = (size_t)64 * 4096 * sizeof(float);  // one batch: up to 64 lines, 16 KB apart
  float* buf;
  uint64_t* o;
  UB_CHECK(hipMalloc(&buf, region * reps * 10));
  UB_CHECK(hipMalloc(&o, 16));
  UB_CHECK(hipMemset(buf, 0, region * reps * 10));
  double t[10];
  int ns[10] = {1, 2, 4, 8, 16, 24, 32, 40, 48, 64};
  size_t off = 0;
  auto next = [&]() { float* p = buf + off / sizeof(float); off += region * reps; return p; };
  t[0] = run<1>(next(), region, reps, o);
  t[1] = run<2>(next(), region, reps, o);
  t[2] = run<4>(next(), region, reps, o);
  t[3] = run<8>(next(), region, reps, o);
  t[4] = run<16>(next(), region, reps, o);
  t[5] = run<24>(next(), region, reps, o);
  t[6] = run<32>(next(), region, reps, o);
  t[7] = run<40>(next(), region, reps, o);
  t[8] = run<48>(next(), region, reps, o);
  t[9] = run<64>(next(), region, reps, o);
  int knee = ns[9];
  for (int i = 0; i < 10; ++i) {
    printf("independent misses %2d : %8.0f cycles per batch (%6.1f per miss)\n", ns[i], t[i], t[i] / ns[i]);
  }
  // the first batch size whose time exceeds 1.6x the single-miss round trip
  for (int i = 1; i < 10; ++i)
    if (t[i] > 1.6 * t[0]) {
      knee = ns[i - 1];
      break;
    }
  printf("# l1_outstanding_misses_per_wave %d\n", knee);
  printf("# hbm_round_trip_cycles %.0f\n", t[0]);
  UB_CHECK(hipFree(buf));
  UB_CHECK(hipFree(o));
  return 0;
}
