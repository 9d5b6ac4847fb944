#!/bin/bash
# Short regression run, the MI355X-native counterpart of the reference's
# travis.sh:9-24 / Jenkinsfile:28-91:
#   build -> traces -> run_simulations (local job manager) -> monitor_func_test
#   (regex pass/fail oracle) -> get_stats -> plot-correlation against the
#   statistics archive -> exact per-kernel regression gate.
# The reference downloads recorded V100 traces; there is no network here, so
# the Rodinia-2.0-ft suite is generated synthetically (same apps, same args
# folders).  Environment:
#   CI_CONFIG  (QV100-SASS)   launch config        CI_WORK (./ci_run) scratch
#   CI_APPS    (all)          comma list of apps   CI_NAME (ci)       launch name
#   CI_GOLDEN  (ci/golden_<CONFIG>_rodinia_2.0-ft.csv)  statistics archive
#   CI_UPDATE=1 re-records the archive instead of checking it
set -euo pipefail
ROOT=$(cd "$(dirname "$0")" && pwd)
cd "$ROOT"
CONFIG=${CI_CONFIG:-QV100-SASS}
WORK=${CI_WORK:-$ROOT/ci_run}
NAME=${CI_NAME:-ci}
APPS=${CI_APPS:-all}
GOLDEN=${CI_GOLDEN:-$ROOT/ci/golden_${CONFIG}_rodinia_2.0-ft.csv}
PY=${PYTHON:-python3}

# 1. build (CPU engine + CLI; the HIP engine too when hipcc is present)
if [ "${CI_SKIP_BUILD:-0}" != "1" ]; then
  $PY build_native.py --cpu-only > "$WORK.build.log" 2>&1 || { cat "$WORK.build.log"; exit 1; }
fi
rm -rf "$WORK"
mkdir -p "$WORK/yml/apps" "$WORK/yml/configs"

# 2. traces in the downloaded-trace layout: <root>/<app>/<args>/traces
$PY - "$WORK" "$APPS" <<'PYEOF'
import os, sys, yaml
sys.path.insert(0, os.getcwd())
from accel_sim_framework_distributed_amd.tracegen import rodinia
work, apps = sys.argv[1], sys.argv[2]
sel = None if apps == "all" else [a if "rodinia" in a else a + "-rodinia-2.0-ft" for a in apps.split(",")]
rodinia.generate_suite(os.path.join(work, "hw_run", "rodinia_2.0-ft"), sel)
# the launch suite: the registry's rodinia_2.0-ft entry, restricted to the selection
reg = yaml.safe_load(open("accel_sim_framework_distributed_amd/job_launching/apps/define-all-apps.yml"))
suite = dict(reg["rodinia_2.0-ft"])
suite["execs"] = [e for e in suite["execs"] if sel is None or next(iter(e)) in sel]
yaml.safe_dump({"rodinia_2.0-ft-ci": suite}, open(os.path.join(work, "yml", "apps", "define-ci.yml"), "w"))
PYEOF
export ASIM_YAML_PATH="$WORK/yml" ASIM_JOB_LOGDIR="$WORK/logs" PROCMAN_STATE="$WORK/procman.json"
export ASIM_CONFIG_ROOT="$WORK/cfgs"

# 3. launch on the local job manager
util/job_launching/run_simulations.py -B rodinia_2.0-ft-ci -C "$CONFIG" -T "$WORK/hw_run/rodinia_2.0-ft" \
  -N "$NAME" -l local -r "$WORK/sim_run"
# 4. wait; non-zero exit on any failed job (exit detected / no Assertion / no deadlock)
util/job_launching/monitor_func_test.py -v -N "$NAME" -r "$WORK/sim_run" -S 1 -T "${CI_TIMEOUT:-1800}" -K \
  -s "$WORK/stats.csv"
# 5. per-kernel statistics
util/job_launching/get_stats.py -k -K -N "$NAME" -r "$WORK/sim_run" > "$WORK/per_kernel.csv"
# 6. correlation against the statistics archive, then the exact gate
if [ "${CI_UPDATE:-0}" = "1" ]; then
  $PY tools/ci_regress.py --stats "$WORK/per_kernel.csv" --record "$GOLDEN"
fi
util/plotting/plot-correlation.py -c "$WORK/per_kernel.csv" -F "$GOLDEN" --clock_mhz 1132 -o "$WORK/correl" \
  -p "$NAME" | tee "$WORK/correl.txt"
SUBSET=""
[ "$APPS" != "all" ] && SUBSET="--subset"
$PY tools/ci_regress.py --stats "$WORK/per_kernel.csv" --check "$GOLDEN" --tolerance "${CI_TOLERANCE:-0}" $SUBSET
echo "travis.sh: all checks passed"
