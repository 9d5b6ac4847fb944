#!/bin/bash
# GPU batch: new tracer tests (allocation snapshots, BBVs, tiny ring), the
# host-streamed trace on the GPU engine, then the RCCL library-kernel counters.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
(python3 -c "import os; print(\"host cpus: affinity\", len(os.sched_getaffinity(0)), \"cpu_count\", os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; nproc) | tee gpurun_out/r4_host_cpus.txt
timeout -k 10 400 python3 -u -m pytest tests/test_isatrace.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_isatrace_tests2.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a gpurun_out/r4_isatrace_tests2.log
tail -15 gpurun_out/r4_isatrace_tests2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 120 --timeout-method thread -k "host_streamed or trace_window" > gpurun_out/r4_hoststream.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a gpurun_out/r4_hoststream.log
tail -8 gpurun_out/r4_hoststream.log
[ $rc -eq 0 ] || exit $rc
bash tools/archive/gpu_r4_rccl.sh
