#!/bin/bash
# On the MI355X box: run the automatically instrumented HIP apps
# (bin/isatrace/<app>, built here by isatrace/build.py from the unmodified
# csrc/apps sources), then count the plain builds' instructions with
# rocprofv3 SQ counters and compare (isatrace/verify.py).  Every GPU step has
# its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/isat
mkdir -p $out
CTR="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
APPS=${ISAT_APPS:-"vectoradd:65536 nn:65536 bfs:8192 hotspot:128,2 pathfinder:20000,8"}
cd /tmp
for spec in $APPS; do
  app=${spec%%:*}; args=$(echo ${spec#*:} | tr ',' ' ')
  echo "== $app $args"
  # streamed through the host ring unless ISAT_BUF_MB asks for a device buffer
  env ASIM_TRACE_DIR=$out/$app ${ISAT_BUF_MB:+ASIM_TRACE_BUF_MB=$ISAT_BUF_MB} timeout -k 10 120 $R/bin/isatrace/$app $args \
    > $out/$app.run.log 2>&1 || { echo "$app traced run failed"; tail -5 $out/$app.run.log; exit 1; }
  tail -2 $out/$app.run.log
  timeout -k 10 120 $R/bin/apps/$app $args > $out/$app.plain.log 2>&1 || { echo "$app plain run failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $out/$app.pmc -o run -- $R/bin/apps/$app $args \
    > $out/$app.pmc.log 2>&1 || { echo "$app pmc failed"; tail -5 $out/$app.pmc.log; exit 1; }
  python3 $R/accel_sim_framework_distributed_amd/isatrace/verify.py $out/$app $out/$app.pmc > $out/$app.verify.txt \
    || { echo "$app verify failed"; exit 1; }
  cat $out/$app.verify.txt
  du -sh $out/$app
  [ -n "$ISAT_KEEP" ] || rm -rf $out/$app $out/$app.pmc  # traces are large; keep the verdicts
done
