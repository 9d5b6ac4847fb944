#!/bin/bash
# bisect a GPU-engine crash seen in the correlation run (nn, tuned MI355X config)
export TMPDIR=/tmp
W=/tmp/repro_$$; mkdir -p $W; cd $W
tar xzf $GRAFT_REPO_ROOT/tools/repro/nn.tgz
OUT=$GRAFT_REPO_ROOT/gpurun_out/repro; mkdir -p $OUT
for v in "base:" "nomall:-sim_mall none" "noxcd:-sim_xcd 0" "neither:-sim_mall none -sim_xcd 0"; do
  name=${v%%:*}; extra=${v#*:}
  timeout -k 5 120 $GRAFT_REPO_ROOT/bin/accel-sim.out -config $GRAFT_REPO_ROOT/tools/repro/nn_gpgpusim.config $extra \
     -trace nn/42764/traces/kernelslist.g > $OUT/$name.out 2> $OUT/$name.err
  rc=$?
  echo "$name rc=$rc $(grep -c '' $OUT/$name.out) lines; $(grep 'gpu_sim_cycle' $OUT/$name.out | tail -1)"
  tail -2 $OUT/$name.err
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 134 ] && [ $rc -ne 139 ]; then break; fi
done
