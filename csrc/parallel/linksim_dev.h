// Device-resident epoch loop of the packet collective: state layout and host
// API (implementation and kernels: linksim_dev.hip; driver loop over RCCL:
// exchange.cc exchange_run_device; in-process multi-rank emulation:
// exchange.cc dev_run_local).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "parallel/linksim.h"

namespace asim {

constexpr int64_t kDlsI64Max = 0x7fffffffffffffffll;

enum : int32_t {
  DLS_RUN = 0,
  DLS_DONE = 1,
  DLS_SPILL = 2,  // an overflow exchange is due (every rank stops at the same epoch)
  DLS_ERR_DST = 3,
  DLS_ERR_SRC = 4,
  DLS_ERR_SPILL = 5,
  DLS_ERR_CAP = 6,
  DLS_ERR_DEADLOCK = 7,
};

enum : int { DLS_MODE_FIRST = 0, DLS_MODE_NEXT = 1, DLS_MODE_SPILL = 2 };

// one rank's LinkSim in HBM (the header of its state block)
struct DlsState {
  LsGeom g;
  uint64_t link_free[kLsMaxLinks];
  uint64_t recv_left, send_left, sent, finish_ps;
  int64_t t, t_end, ann_next, ann_busy;
  uint64_t epochs, packets;
  int64_t extra_total;  // overflow words packed in the last epoch
  int64_t lheap_off[kLsMaxLinks];  // per-link pending-send heaps: offset (items), size, capacity
  int32_t lheap_n[kLsMaxLinks];
  int32_t lheap_cap[kLsMaxLinks];
  int32_t status;
  int32_t k, hdr;
  int32_t pad;
  uint64_t prof[8];  // epoch kernel shader clocks, summed: load, unpack, pack, store | pack: emit, reductions, slots
};

// byte offsets inside one rank's state block
struct DlsLayout {
  size_t bytes = 0;
  size_t off_heap = 0, off_pk = 0, off_extra = 0, off_ew = 0, off_cnt = 0, off_fill = 0;
  int64_t cap = 0;
};

DlsLayout dls_layout(int world, int64_t cap);
int64_t dls_capacity(const LinkSim::Export& e);
// the state block of `e` (L.bytes bytes at img)
void dls_image(const LinkSim::Export& e, const DlsLayout& L, int k, int hdr, char* img);
// one epoch of `nranks` state blocks (block b at states + b * L.bytes):
// FIRST packs the first epoch at *t0; NEXT delivers the received slots and
// packs the next epoch; SPILL does the same with the overflow words
// (rank b's at spill + spill_off[b] .. spill_off[b + 1]).  Rank b receives its
// slot from source r at recv + b * recv_rank_stride + r * recv_src_stride and
// packs into send + b * send_rank_stride.
void dls_launch_epoch(char* states, const DlsLayout& L, int nranks, const int64_t* recv, int64_t recv_src_stride,
                      int64_t recv_rank_stride, int64_t* send, int64_t send_rank_stride, const int64_t* spill,
                      const int64_t* spill_off, const int64_t* t0, int mode, void* stream);
// send [s][d][slot] -> recv [d][s][slot] (the emulation's all-to-all)
void dls_launch_transpose(const int64_t* send, int64_t* recv, int world, int slot, void* stream);
const char* dls_status_name(int32_t st);

}  // namespace asim
