#!/bin/bash
# Round 5: ISA-tracer GPU tests for device-function calls and the binary-only
# path, then the power refit with the issue-weighted static column
# (tools/archive/gpu_r5_power2.sh).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r5c17
mkdir -p $out
cd $R && timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_isatrace.py -k "binary_path or device_function" > $out/pytest_isatrace_calls.log 2>&1; e=$?
tail -4 $out/pytest_isatrace_calls.log
[ $e -eq 0 ] || exit $e
bash $R/tools/archive/gpu_r5_power2.sh
