#!/bin/bash
# A/B/A/B of the node bench in one call: widen() with and without the second
# doubling of a critical application's host thread team (ASIM_NODE_WIDEN_WIDER)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/widen
mkdir -p $O
for i in 1 2; do
  for w in 1 0; do
    ASIM_NODE_WIDEN_WIDER=$w timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/bench_w${w}_$i.json 2> $O/bench_w${w}_$i.err \
      || { tail $O/bench_w${w}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_w${w}_$i.json')); c=d['config']; print('wider=$w', d['value'], d['ms_per_step'], c.get('node_cpu_threads'), d['gpu_engine']['insn_share'])"
  done
done
