#!/bin/bash
# two GPU-engine simulations of the MI355X config at once on one GPU
export TMPDIR=/tmp
W=/tmp/repro_$$; mkdir -p $W; cd $W
tar xzf $GRAFT_REPO_ROOT/tools/repro/nn.tgz
OUT=$GRAFT_REPO_ROOT/gpurun_out/repro_conc; mkdir -p $OUT
for i in 1 2; do
  timeout -k 5 100 $GRAFT_REPO_ROOT/bin/accel-sim.out -config $GRAFT_REPO_ROOT/tools/repro/nn_gpgpusim.config \
     -trace nn/42764/traces/kernelslist.g > $OUT/p$i.out 2> $OUT/p$i.err &
done
wait
for i in 1 2; do echo "p$i: $(grep -c '' $OUT/p$i.out) lines; $(grep 'gpu_sim_cycle\|gpu_sim_insn' $OUT/p$i.out | tr '\n' ' ')"; tail -2 $OUT/p$i.err; done
