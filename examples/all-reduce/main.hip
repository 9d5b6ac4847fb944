// UB_LIBS: -lrccl
// examples/all-reduce for MI355X: the reference's NCCL example
// (examples/all-reduce/main.cu: test_kernel before and after an ncclAllReduce
// of 32 Mi floats per device inside a group, ncclCommInitAll over the local
// devices) written against RCCL.  Kernels carry asim_trace annotations, so
//   ASIM_TRACE_DIR=<dir> ROCP_TOOL_LIBRARIES=bin/libasim_tracer.so ./all-reduce
// produces a kernelslist.g with both kernels and the collective -- with its
// count / datatype / op / communicator size recorded by the rocprofiler-sdk
// tool (the reference's interposer drops them) -- ready for
// `-collective_model packet` simulation.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../csrc/tracer/asim_trace.h"

using namespace asim_trace;

#define RCCL_CHECK(x)                                                               \
  do {                                                                              \
    ncclResult_t r_ = (x);                                                          \
    if (r_ != ncclSuccess) {                                                        \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

template <class TR>
__global__ void test_kernel(TR tr, int* ptr) {
  auto w = tr.wave();
  ASIM_VALU(w, V_LSHLREV_B32, 1, 0);
  ASIM_ST(w, GLOBAL_STORE_DWORD, ptr + threadIdx.x, 7, 2, 1);
  w.exit();
}

int main(int argc, char** argv) {
  int ndev = 0;
  ASIM_HIP(hipGetDeviceCount(&ndev));
  if (argc > 1) ndev = std::min(ndev, atoi(argv[1]));
  const size_t count = 32u * 1024u * 1024u;
  std::vector<int> devs(ndev);
  std::vector<float*> send(ndev), recv(ndev);
  std::vector<int*> scratch(ndev);
  std::vector<hipStream_t> st(ndev);
  for (int i = 0; i < ndev; ++i) {
    devs[i] = i;
    ASIM_HIP(hipSetDevice(i));
    ASIM_HIP(hipMalloc(&send[i], count * sizeof(float)));
    ASIM_HIP(hipMalloc(&recv[i], count * sizeof(float)));
    ASIM_HIP(hipMalloc(&scratch[i], 256 * sizeof(int)));
    ASIM_HIP(hipStreamCreate(&st[i]));
    std::vector<float> h(count, 3.14f * (1 + i));
    memcpy_htod(send[i], h.data(), count * sizeof(float));
  }
  std::vector<ncclComm_t> comms(ndev);
  RCCL_CHECK(ncclCommInitAll(comms.data(), ndev, devs.data()));
  for (int i = 0; i < ndev; ++i) {
    ASIM_HIP(hipSetDevice(i));
    launch("_Z11test_kernelPi", test_kernel<On>, test_kernel<Off>, dim3(1), dim3(256), 0, st[i], scratch[i]);
  }
  RCCL_CHECK(ncclGroupStart());
  for (int i = 0; i < ndev; ++i)
    RCCL_CHECK(ncclAllReduce(send[i], recv[i], count, ncclFloat, ncclSum, comms[i], st[i]));
  RCCL_CHECK(ncclGroupEnd());
  for (int i = 0; i < ndev; ++i) {
    ASIM_HIP(hipSetDevice(i));
    ASIM_HIP(hipStreamSynchronize(st[i]));
    launch("_Z11test_kernelPi", test_kernel<On>, test_kernel<Off>, dim3(1), dim3(256), 0, st[i], scratch[i]);
  }
  float expect = 0;
  for (int i = 0; i < ndev; ++i) expect += 3.14f * (1 + i);
  bool ok = true;
  for (int i = 0; i < ndev; ++i) {
    float v = 0;
    ASIM_HIP(hipSetDevice(i));
    ASIM_HIP(hipMemcpy(&v, recv[i] + count / 2, sizeof(float), hipMemcpyDeviceToHost));
    ok = ok && std::fabs(v - expect) < 1e-3f * expect;
  }
  for (int i = 0; i < ndev; ++i) {
    RCCL_CHECK(ncclCommDestroy(comms[i]));
    ASIM_HIP(hipSetDevice(i));
    ASIM_HIP(hipFree(send[i]));
    ASIM_HIP(hipFree(recv[i]));
    ASIM_HIP(hipFree(scratch[i]));
  }
  printf("all-reduce over %d device(s): %s\n", ndev, ok ? "PASSED" : "FAILED");
  return ok ? 0 : 1;
}
