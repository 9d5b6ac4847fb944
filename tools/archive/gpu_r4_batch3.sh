#!/bin/bash
# GPU batch: the full GPU-engine test file (trace windows on the shared
# TraceWindows, host streaming, in-kernel power sampler), the MFMA counters of
# engine_kernel with power sampling on, then app phase times and the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_engine.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_gpu_engine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/power_run.py --app hotspot > $O/power_run.log 2>&1
rc=$?; echo "power run rc=$rc"; cat $O/power_run.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 rocprofv3 -L > $O/counters_avail.txt 2>&1
MF=$(grep -o "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*" $O/counters_avail.txt | sort -u | head -4 | tr '\n' ' ')
echo "mfma counters: $MF"
if [ -n "$MF" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $MF SQ_WAVES --kernel-trace -d $O/pmc_mfma -o run -- python3 tools/power_run.py --app hotspot > $O/pmc_mfma.log 2>&1
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python3 -u tools/app_phases.py --apps hotspot,backprop,heartwall,bfs,srad_v2,streamcluster,nw,lud,pathfinder,nn \
  --engines gpu,cpu --threads 1,2,4 --reps 2 --out $O/app_phases.json > $O/app_phases.log 2>&1
rc=$?; echo "phases rc=$rc"; tail -3 $O/app_phases.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log; exit $rc
