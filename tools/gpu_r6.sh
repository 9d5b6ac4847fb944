#!/bin/bash
# Round-6 GPU runner, one parameterised script (replaces the per-call
# gpu_r5_*.sh one-shots).  usage: bash tools/gpu_r6.sh <step> [<step> ...]
#   state   : pytest of the global-state engine (GPU == CPU), one-SM wall time
#             of both state builds, GPU-only bench of both builds
#   tests   : the whole GPU suite
#   bench   : bench.py (node) + rocprofv3 kernel stats
# Every GPU step runs under its own timeout; the first failure ends the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6
mkdir -p $O
PT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step_state() {
  ASIM_GPU_STATE=global timeout -k 10 600 $PT tests/test_gpu_engine.py tests/test_icnt.py -k "global_state or rodinia_app or snapshot or pool or back_pressure or router_model_gpu" \
    > $O/pytest_global.log 2>&1 || { tail -30 $O/pytest_global.log; return 1; }
  tail -3 $O/pytest_global.log
  for app in hotspot bfs; do
    for mode in lds global; do
      echo -n "$mode " >> $O/one_sm.txt
      ASIM_GPU_STATE=$mode ASIM_GPU_PROFILE=0 timeout -k 10 120 python3 tools/engine_pmc_1sm.py --app $app 2>&1 \
        | grep -v amdgpu.ids >> $O/one_sm.txt || return 1
    done
  done
  cat $O/one_sm.txt
  for mode in lds global; do
    ASIM_GPU_STATE=$mode timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 \
      > $O/bench_gpu_$mode.json 2> $O/bench_gpu_$mode.err || { tail $O/bench_gpu_$mode.err; return 1; }
    python3 -c "import json,sys; d=json.load(open('$O/bench_gpu_$mode.json')); print('$mode', d['value'], d['ms_per_step'])"
  done
}
step_tests() {
  timeout -k 10 1000 $PT tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; return 1; }
  tail -3 $O/pytest_gpu.log
}
step_bench() {
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/bench_node.json 2> $O/bench_node.err || { tail $O/bench_node.err; return 1; }
  cat $O/bench_node.json
}
for s in "$@"; do
  echo "== $s"
  step_$s || exit 1
done
