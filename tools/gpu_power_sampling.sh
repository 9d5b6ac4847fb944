#!/bin/bash
# Cost of power sampling on the MI355X engine: one hotspot-sized run with
# -power_simulation_enabled at a 500-cycle sample period under rocprofv3
# kernel tracing; tools/rocpd_summary.py gives the engine kernel's time and
# launch count, the wall time the rest (the host side of every sample).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/psample
mkdir -p $out
python3 -c "
from accel_sim_framework_distributed_amd.tracegen import rodinia
from accel_sim_framework_distributed_amd.power import xmlcfg
rodinia.write_app('$out/hs', rodinia.hotspot(1024, 2, 2))
xmlcfg.write_xml('$out/aw.xml', xmlcfg.default_params('QV100'))
"
ARGS="$(python3 -c "from accel_sim_framework_distributed_amd.models import presets; print(' '.join(presets.args_for('QV100')))") -trace $out/hs/kernelslist.g -sim_engine gpu"
cd /tmp
for mode in off on; do
  extra=""
  [ $mode = on ] && extra="-power_simulation_enabled 1 -accelwattch_xml_file $out/aw.xml -gpgpu_runtime_stat 500:0 -power_report_file $out/p.log"
  t0=$(date +%s.%N)
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof_$mode -o run -- \
    $R/bin/accel-sim.out $ARGS $extra > $out/sim_$mode.log 2>&1
  python3 -c "import sys; print(round($(date +%s.%N) - $t0, 3))" > $out/wall_$mode.txt
  python3 $R/tools/rocpd_summary.py $(find $out/prof_$mode -name "*.db" | head -1) > $out/kstats_$mode.csv
  echo "== power sampling $mode: wall $(cat $out/wall_$mode.txt) s"; head -2 $out/kstats_$mode.csv
  grep -E "^gpu_tot_sim_cycle|gpgpu_simulation_time" $out/sim_$mode.log | tail -2
done
