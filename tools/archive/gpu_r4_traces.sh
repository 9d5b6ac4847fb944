#!/bin/bash
# Round 4: capture the Rodinia HIP suite's ISA traces + rocprofv3 timings and
# counters on the MI355X, and bring the traces back for local re-simulation
# (tools/local_correlate.py) of model changes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_trace_and_time.sh || exit 1
out=gpurun_out/corr
tar czf $out/traces.tgz -C $out traces && du -m $out/traces.tgz
sz=$(du -m $out/traces.tgz | cut -f1)
if [ "$sz" -gt 56 ]; then
  rm -f $out/traces.tgz; mkdir -p $out/trace_tgz
  for d in $out/traces/*/; do a=$(basename $d); tar czf $out/trace_tgz/$a.tgz -C $out/traces $a
    s2=$(du -m $out/trace_tgz/$a.tgz | cut -f1); [ "$s2" -gt 8 ] && rm -f $out/trace_tgz/$a.tgz && echo "$a dropped ($s2 MB)"; done
fi
rm -rf $out/traces
du -sh $out
