#!/bin/bash
# quick GPU check of the tree: engine tests, one-SM stage profile (hotspot),
# GPU-engine-only bench.  usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6; T=${1:-quick}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_model_options.py -m gpu \
  > $O/pytest_$T.log 2>&1 || { tail -30 $O/pytest_$T.log; exit 1; }
tail -2 $O/pytest_$T.log
ASIM_GPU_PROFILE=1 timeout -k 10 180 python3 tools/engine_pmc_1sm.py --app hotspot > $O/stage_$T.log 2>&1 || { tail $O/stage_$T.log; exit 1; }
grep -E "iss\.|issue|clocks each|sms=" $O/stage_$T.log
timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 > $O/bench_gpu_$T.json 2> $O/bench_gpu_$T.err || { tail $O/bench_gpu_$T.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_gpu_$T.json')); print('gpu-only', d['value'], d['ms_per_step'])"
