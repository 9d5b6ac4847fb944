#!/bin/bash
# Round-3 GPU batch on the MI355X box:
#  1. launch overheads as rocprofv3 sees them: isolated (after an event),
#     queued, idle-queue and back-to-back chains (ub_launch + launch_latency.py)
#  2. GPU==CPU bit-exactness of the new memory-hierarchy / DVFS paths
#  3. instruction-count verify records of the six apps not yet covered
#  4. power validation: 30 kernels, socket power + graphics clock + rail
#     voltage + the power limit from amd-smi, ISA traces, DVFS-aware fit
# Every GPU step has its own time limit; the script stops at the first failure.
# Usage: gpu_r3b.sh a   (steps 1-3)   |   gpu_r3b.sh b   (step 4)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r3b
mkdir -p $out
cd /tmp
if [ "${1:-a}" = a ]; then
echo "== launch overheads"
timeout -k 10 240 python3 $R/accel_sim_framework_distributed_amd/hw_stats/launch_latency.py -o $out/launch_rocprof \
  > $out/launch.log 2>&1 || { echo "launch_latency failed"; tail -5 $out/launch.log; exit 1; }
tail -22 $out/launch.log
echo "== GPU engine bit-exactness (new paths)"
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_checkpoint.py -m gpu -x -q --timeout 180 \
  --timeout-method thread -k "xcd_release or xcd_mall or checkpoint or mi355x" > $out/gputest.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $out/gputest.log; exit 1; }
tail -3 $out/gputest.log
cd /tmp
echo "== isatrace verify, six more apps"
ISAT_APPS="backprop:4096 heartwall:1,51 lud:64 nw:128,10 srad_v2:128,128,0.5,2 streamcluster:1024,16,24,6" \
  timeout -k 10 900 bash $R/tools/gpu_isatrace.sh > $out/isat.log 2>&1 || { echo "isatrace failed"; tail -20 $out/isat.log; exit 1; }
grep -E "^==|MATCH|match|mismatch|total" $out/isat.log | head -40
cp -r $R/gpurun_out/isat/*.verify.txt $out/ 2>/dev/null
exit 0
fi
echo "== power validation"
PWR_SIM_SECS=700 timeout -k 10 1000 bash $R/tools/gpu_power.sh > $out/power.log 2>&1; e=$?
tail -40 $out/power.log
exit $e
