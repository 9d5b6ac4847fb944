#!/bin/bash
# rocprofv3 counters of the all-reduce example's library kernels (RCCL on a
# 1-rank communicator: the HIP runtime's copy / fill blit kernels), two PMC
# passes; tools/rccl_validate.py compares them with the simulator's
# collective copy-kernel stand-in.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4rccl
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $OUT/p1 -o p1 -- bin/examples/all-reduce > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc TCC_REQ_sum TCC_HIT_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $OUT/p2 -o p2 -- bin/examples/all-reduce > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $OUT/p3 -o p3 -- bin/examples/all-reduce > $OUT/p3.log 2>&1
echo rccl-pmc-done
