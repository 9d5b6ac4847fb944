// UB_LIBS: -lrccl
// Which RCCL device kernels run on a one-GPU communicator?  Every collective
// and a send / receive pair to the rank itself, each once, on one device; run
// under rocprofv3 --kernel-trace to list the kernels (tools/gpu_r5_rccl_self.sh).
// On one rank RCCL may satisfy a collective with a runtime copy instead of its
// own kernel; the point-to-point self exchange goes through its kernel.
#include <rccl/rccl.h>

#include <cstdio>
#include <vector>

#include "../../csrc/apps/app_common.h"

#define RCCL_CHECK(x)                                                                            \
  do {                                                                                           \
    ncclResult_t r_ = (x);                                                                       \
    if (r_ != ncclSuccess) {                                                                     \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      return 1;                                                                                  \
    }                                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const size_t count = argc > 1 ? (size_t)atol(argv[1]) : (size_t)1 << 20;
  int dev = 0;
  ncclComm_t comm;
  RCCL_CHECK(ncclCommInitAll(&comm, 1, &dev));
  hipStream_t st;
  APP_HIP(hipSetDevice(0));
  APP_HIP(hipStreamCreate(&st));
  float *a, *b;
  APP_HIP(hipMalloc(&a, count * sizeof(float)));
  APP_HIP(hipMalloc(&b, count * sizeof(float)));
  std::vector<float> h(count, 1.0f);
  APP_HIP(hipMemcpy(a, h.data(), count * sizeof(float), hipMemcpyHostToDevice));
  RCCL_CHECK(ncclAllReduce(a, b, count, ncclFloat, ncclSum, comm, st));
  RCCL_CHECK(ncclAllReduce(a, a, count, ncclFloat, ncclSum, comm, st));
  RCCL_CHECK(ncclBroadcast(a, b, count, ncclFloat, 0, comm, st));
  RCCL_CHECK(ncclAllGather(a, b, count, ncclFloat, comm, st));
  RCCL_CHECK(ncclReduceScatter(a, b, count, ncclFloat, ncclSum, comm, st));
  RCCL_CHECK(ncclAllToAll(a, b, count, ncclFloat, comm, st));
  RCCL_CHECK(ncclGroupStart());
  RCCL_CHECK(ncclSend(a, count, ncclFloat, 0, comm, st));
  RCCL_CHECK(ncclRecv(b, count, ncclFloat, 0, comm, st));
  RCCL_CHECK(ncclGroupEnd());
  APP_HIP(hipStreamSynchronize(st));
  APP_HIP(hipMemcpy(h.data(), b, sizeof(float) * 4, hipMemcpyDeviceToHost));
  printf("rccl-self: %zu floats, b[0] = %.1f\n", count, h[0]);
  APP_HIP(hipFree(a));
  APP_HIP(hipFree(b));
  ncclCommDestroy(comm);
  return 0;
}
