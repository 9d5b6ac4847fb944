// UB_LIBS: -lrccl
// examples/all-reduce for MI355X: the reference's NCCL example
// (examples/all-reduce/main.cu: test_kernel before and after an ncclAllReduce
// of 32 Mi floats per device inside a group, ncclCommInitAll over the local
// devices) written against RCCL, plain HIP.  Its automatically instrumented
// build (bin/isatrace/all-reduce, isatrace/build.py) run as
//   ASIM_TRACE_DIR=<dir> ROCP_TOOL_LIBRARIES=bin/libasim_tracer.so bin/isatrace/all-reduce
// produces a kernelslist.g with both kernels' ISA traces and the collective --
// with its count / datatype / op / communicator size recorded by the
// rocprofiler-sdk tool (the reference's interposer drops them) -- ready for
// `-collective_model packet` simulation.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../csrc/apps/app_common.h"

#define RCCL_CHECK(x)                                                               \
  do {                                                                              \
    ncclResult_t r_ = (x);                                                          \
    if (r_ != ncclSuccess) {                                                        \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ void test_kernel(int* ptr) { ptr[threadIdx.x] = 7; }

int main(int argc, char** argv) {
  int ndev = 0;
  APP_HIP(hipGetDeviceCount(&ndev));
  if (argc > 1) ndev = std::min(ndev, atoi(argv[1]));
  const size_t count = 32u * 1024u * 1024u;
  std::vector<int> devs(ndev);
  std::vector<float*> send(ndev), recv(ndev);
  std::vector<int*> scratch(ndev);
  std::vector<hipStream_t> st(ndev);
  for (int i = 0; i < ndev; ++i) {
    devs[i] = i;
    APP_HIP(hipSetDevice(i));
    APP_HIP(hipMalloc(&send[i], count * sizeof(float)));
    APP_HIP(hipMalloc(&recv[i], count * sizeof(float)));
    APP_HIP(hipMalloc(&scratch[i], 256 * sizeof(int)));
    APP_HIP(hipStreamCreate(&st[i]));
    std::vector<float> h(count, 3.14f * (1 + i));
    APP_HIP(hipMemcpy(send[i], h.data(), count * sizeof(float), hipMemcpyHostToDevice));
  }
  std::vector<ncclComm_t> comms(ndev);
  RCCL_CHECK(ncclCommInitAll(comms.data(), ndev, devs.data()));
  for (int i = 0; i < ndev; ++i) {
    APP_HIP(hipSetDevice(i));
    test_kernel<<<1, 256, 0, st[i]>>>(scratch[i]);
  }
  RCCL_CHECK(ncclGroupStart());
  for (int i = 0; i < ndev; ++i)
    RCCL_CHECK(ncclAllReduce(send[i], recv[i], count, ncclFloat, ncclSum, comms[i], st[i]));
  RCCL_CHECK(ncclGroupEnd());
  for (int i = 0; i < ndev; ++i) {
    APP_HIP(hipSetDevice(i));
    APP_HIP(hipStreamSynchronize(st[i]));
    test_kernel<<<1, 256, 0, st[i]>>>(scratch[i]);
  }
  float expect = 0;
  for (int i = 0; i < ndev; ++i) expect += 3.14f * (1 + i);
  bool ok = true;
  for (int i = 0; i < ndev; ++i) {
    float v = 0;
    APP_HIP(hipSetDevice(i));
    APP_HIP(hipMemcpy(&v, recv[i] + count / 2, sizeof(float), hipMemcpyDeviceToHost));
    ok = ok && std::fabs(v - expect) < 1e-3f * expect;
  }
  for (int i = 0; i < ndev; ++i) {
    RCCL_CHECK(ncclCommDestroy(comms[i]));
    APP_HIP(hipSetDevice(i));
    APP_HIP(hipFree(send[i]));
    APP_HIP(hipFree(recv[i]));
    APP_HIP(hipFree(scratch[i]));
  }
  printf("all-reduce over %d device(s): %s\n", ndev, ok ? "PASSED" : "FAILED");
  return ok ? 0 : 1;
}
