#!/bin/bash
# Round-6 GPU runner, one parameterised script (replaces the per-call
# gpu_r5_*.sh one-shots).  usage: bash tools/gpu_r6.sh <step> [<step> ...]
#   state   : pytest of the global-state engine (GPU == CPU), one-SM wall time
#             of both state builds, GPU-only bench of both builds
#   tests   : the whole GPU suite
#   bench   : bench.py (node) + rocprofv3 kernel stats
#   devloop : device-resident collective epoch loop: GPU tests + per-epoch cost
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
step_batch() {
  ASIM_GPU_STATE=global timeout -k 10 600 $PT tests/test_gpu_engine.py -k "global_state or batch or pool or resources" \
    > $O/pytest_batch.log 2>&1 || { tail -30 $O/pytest_batch.log; return 1; }
  tail -3 $O/pytest_batch.log
  for mode in lds global; do
    ASIM_GPU_STATE=$mode timeout -k 10 600 python3 bench.py --sweep --engine gpu --steps 1 --warmup 0 \
      > $O/sweep_gpu_$mode.json 2> $O/sweep_gpu_$mode.err || { tail $O/sweep_gpu_$mode.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/sweep_gpu_$mode.json')); print('sweep $mode', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'))"
  done
  ASIM_GPU_STATE=global timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 \
    > $O/bench_gpu_global_batch.json 2> $O/bench_gpu_global_batch.err || { tail $O/bench_gpu_global_batch.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_gpu_global_batch.json')); print('gpu global batch', d['value'], d['ms_per_step'])"
}
step_scaling() {
  for st in lds global; do
    for app in hotspot bfs; do
      ASIM_GPU_STATE=$st timeout -k 10 300 python3 tools/batch_scaling.py --app $app --n ${NS:-1,2,3,4,6} \
        2>&1 | grep -v amdgpu.ids >> $O/scaling.jsonl || return 1
    done
  done
  cat $O/scaling.jsonl
}
step_scaling2() {
  # global-state batch launches with the concurrent-batch launcher, 3 and 4 blocks per CU
  for bpc in ${BPCS:-2 3}; do
    for app in hotspot bfs; do
      ASIM_GPU_BLOCKS_PER_CU=$bpc ASIM_GPU_STATE=global timeout -k 10 300 python3 tools/batch_scaling.py --app $app \
        --n ${NS:-1,2,4,6,8} 2>&1 | grep -v amdgpu.ids | sed "s/^{/{\"bpc\": $bpc, /" >> $O/scaling2.jsonl || return 1
    done
  done
  cat $O/scaling2.jsonl
}
step_sweep_global() {
  for bpc in ${BPCS:-2 3}; do
    ASIM_GPU_BLOCKS_PER_CU=$bpc ASIM_GPU_STATE=global timeout -k 10 300 python3 bench.py --sweep --engine gpu --steps 1 \
      --warmup 0 > $O/sweep_gpu_global_bpc$bpc.json 2> $O/sweep_gpu_global_bpc$bpc.err || { tail -3 $O/sweep_gpu_global_bpc$bpc.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/sweep_gpu_global_bpc$bpc.json')); print('sweep global bpc $bpc', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'))"
  done
}
step_pmc_scaling() {
  # L2 hit rate of the global-state engine with 1 and 4 simulations at once
  for n in 1 4; do
    ASIM_GPU_STATE=global timeout -s KILL 120 rocprofv3 --kernel-trace --stats \
      --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/pmc_n$n -o pmc -- \
      python3 tools/batch_scaling.py --app hotspot --n $n > $O/pmc_n$n.log 2>&1 || { tail $O/pmc_n$n.log; return 1; }
    db=$(find $O/pmc_n$n -name "*.db" | head -1)
    python3 tools/pmc_summary.py "$db" engine_batch_kernel > $O/pmc_n$n.json && cat $O/pmc_n$n.json
  done
}
step_diag() {
  ASIM_GPU_STATE=global timeout -k 10 120 python3 -c "
import torch, sys; sys.path.insert(0, '.')
from accel_sim_framework_distributed_amd import _native
m = _native.load(prefer_torch_runtime=True); print(m.gpu_batch_stats(), m.gpu_cus_per_sim(80, 32), m.gpu_cu_count())" \
    2>&1 | grep -v amdgpu.ids
}
step_split() {
  timeout -k 10 600 $PT tests/test_gpu_engine.py -k "split or global_state or batch or resources or rodinia_app" \
    > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; return 1; }
  tail -3 $O/pytest_split.log
  timeout -k 10 60 python3 -c "
import torch, sys, json; sys.path.insert(0, '.')
from accel_sim_framework_distributed_amd import _native
m = _native.load(prefer_torch_runtime=True); print(json.dumps(m.gpu_engine_modes()))" 2>&1 | grep -v amdgpu.ids | tee $O/engine_modes.json
  for app in hotspot bfs; do
    for mode in lds split; do
      echo -n "$mode " >> $O/one_sm_split.txt
      ASIM_GPU_STATE=$mode ASIM_GPU_PROFILE=0 timeout -k 10 120 python3 tools/engine_pmc_1sm.py --app $app 2>&1 \
        | grep -v amdgpu.ids >> $O/one_sm_split.txt || return 1
    done
  done
  cat $O/one_sm_split.txt
  for app in hotspot bfs; do
    ASIM_GPU_STATE=split timeout -k 10 300 python3 tools/batch_scaling.py --app $app --n ${NS:-1,2,3,4,6} 2>&1 \
      | grep -v amdgpu.ids >> $O/scaling_split.jsonl || return 1
  done
  cat $O/scaling_split.jsonl
  for what in "--engine gpu --steps 2 --warmup 1" "--sweep --engine gpu --steps 1 --warmup 0"; do
    tag=$(echo $what | awk '{print ($1=="--sweep")?"sweep":"bench"}')
    ASIM_GPU_STATE=split timeout -k 10 400 python3 bench.py $what > $O/${tag}_gpu_split.json 2> $O/${tag}_gpu_split.err \
      || { tail -3 $O/${tag}_gpu_split.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/${tag}_gpu_split.json')); print('$tag split', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'))"
  done
}
step_split2() {
  # split-state build with batch launches: tests, concurrency scaling, GPU-only suite and sweep, node bench
  ASIM_GPU_STATE=split timeout -k 10 600 $PT tests/test_gpu_engine.py -k "split or batch or rodinia_app" \
    > $O/pytest_split2.log 2>&1 || { tail -30 $O/pytest_split2.log; return 1; }
  tail -3 $O/pytest_split2.log
  for app in hotspot bfs; do
    ASIM_GPU_STATE=split timeout -k 10 300 python3 tools/batch_scaling.py --app $app --n ${NS:-1,2,3,4,6,8} 2>&1 \
      | grep -v amdgpu.ids >> $O/scaling_split_batch.jsonl || return 1
  done
  cat $O/scaling_split_batch.jsonl
  for what in "--engine gpu --steps 2 --warmup 1" "--sweep --engine gpu --steps 1 --warmup 0" "--steps 10 --warmup 3"; do
    tag=$(echo $what | awk '{print ($1=="--sweep")?"sweep_gpu":($1=="--engine")?"bench_gpu":"bench_node"}')
    ASIM_GPU_STATE=split timeout -k 10 400 python3 bench.py $what > $O/${tag}_split_batch.json 2> $O/${tag}_split_batch.err \
      || { tail -3 $O/${tag}_split_batch.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/${tag}_split_batch.json')); print('$tag split+batch', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'), d.get('gpu_engine',{}).get('insn_share'))"
  done
}
step_nodecmp() {
  # node bench, GPU-only suite and sweep: LDS-state vs split-state engine, same box
  for st in lds split; do
    for what in "--steps 10 --warmup 3" "--engine gpu --steps 2 --warmup 1" "--sweep --engine gpu --steps 1 --warmup 0"; do
      tag=$(echo $what | awk '{print ($1=="--sweep")?"sweep_gpu":($1=="--engine")?"bench_gpu":"bench_node"}')
      ASIM_GPU_STATE=$st timeout -k 10 400 python3 bench.py $what > $O/${tag}_$st.json 2> $O/${tag}_$st.err \
        || { tail -3 $O/${tag}_$st.err; return 1; }
      python3 -c "import json; d=json.load(open('$O/${tag}_$st.json')); print('$tag $st', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'), d.get('gpu_engine',{}).get('insn_share'))"
    done
  done
}
step_corr_gpu() {
  # the round-5 correlation capture (ISA traces + rocprofv3 timings, corr_data/) simulated with the tuned
  # MI355X config on the GPU engine and on the host engine: speed and cycle MAE of the same simulations
  for eng in gpu cpu; do
    cfg=MI355X_TUNED; [ $eng = gpu ] && cfg=MI355X_TUNED-GPU_ENGINE
    t0=$(date +%s.%N)
    CORR_SRC=$GRAFT_REPO_ROOT/corr_data CFG=$cfg JOBS=${CORR_JOBS:-2} timeout -k 10 900 \
      bash tools/local_full_correlate.sh /tmp/corr_$eng > $O/corr_$eng.log 2>&1 || { tail $O/corr_$eng.log; return 1; }
    t1=$(date +%s.%N)
    python3 tools/corr_speed.py /tmp/corr_$eng/simrun /tmp/corr_$eng/correl $(python3 -c "print($t1 - $t0)") $eng \
      | tee -a $O/corr_speed.jsonl
    cp /tmp/corr_$eng/correl/mi355x-summary.json $O/corr_${eng}_summary.json
  done
}
step_nodetol() {
  # node bench (split build) at several makespan tolerances for moving apps onto the GPU engine
  for tol in ${TOLS:-0 0.03 0.08}; do
    ASIM_NODE_GPU_TOLERANCE=$tol timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $O/bench_node_tol$tol.json \
      2> $O/bench_node_tol$tol.err || { tail -3 $O/bench_node_tol$tol.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/bench_node_tol$tol.json')); print('tol $tol', d['value'], d['ms_per_step'], d['gpu_engine']['insn_share'], d['config']['node_predicted_step_ms'])"
  done
}
step_prof() {
  # rocprofv3 kernel statistics of the GPU-engine-only suite (every app on the split-state engine)
  # and of the node bench
  for what in "--engine gpu --steps 2 --warmup 1" "--steps 3 --warmup 1"; do
    tag=$(echo $what | awk '{print ($1=="--engine")?"gpu":"node"}')
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$tag \
      -o run -- python3 $GRAFT_REPO_ROOT/bench.py $what > $GRAFT_REPO_ROOT/$O/prof_$tag.log 2>&1) \
      || { tail -5 $O/prof_$tag.log; return 1; }
    grep '^{"metric"' $O/prof_$tag.log | cut -c1-160
    cat $(find $O/prof_$tag -name "*kernel_stats.csv" | head -1) | cut -c1-160 | head -8
  done
}
step_sweep_node() {
  timeout -k 10 400 python3 bench.py --sweep --steps 1 --warmup 0 > $O/sweep_node.json 2> $O/sweep_node.err \
    || { tail -3 $O/sweep_node.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/sweep_node.json')); print('sweep node', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'), d['config'].get('cpu_slots'), d['gpu_engine'])"
}
step_stage() {
  # one-SM stage profile (profiling build) of the default split engine, bfs and hotspot, plus SQ counters
  for app in ${APPS:-bfs hotspot}; do
    ASIM_GPU_PROFILE=1 timeout -k 10 180 python3 tools/engine_pmc_1sm.py --app $app > $O/stage_$app.log 2>&1 || return 1
    grep -v amdgpu.ids $O/stage_$app.log | head -64
  done
  cs="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $cs -d $GRAFT_REPO_ROOT/$O/pmc_split_bfs -o pmc -- \
    python3 $GRAFT_REPO_ROOT/tools/engine_pmc_1sm.py --app bfs > $GRAFT_REPO_ROOT/$O/pmc_split_bfs.log 2>&1) || return 1
  python3 tools/pmc_summary.py $(find $O/pmc_split_bfs -name "*.db" | head -1) engine_kernel | tee $O/pmc_split_bfs.json
}
step_queues() {
  # hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4): kernels of
  # more streams than queues share a queue and run one after another
  for q in 4 8 12; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python3 tools/batch_scaling.py --app hotspot --n 4,6,8 > $O/queues_scaling_q$q.jsonl 2> $O/queues_q$q.err || { tail $O/queues_q$q.err; return 1; }
    cat $O/queues_scaling_q$q.jsonl
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 > $O/queues_bench_gpu_q$q.json 2>> $O/queues_q$q.err || { tail $O/queues_q$q.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/queues_bench_gpu_q$q.json')); print('q$q gpu-only', d['value'], d['ms_per_step'])"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python3 bench.py --sweep --engine gpu --steps 1 --warmup 0 > $O/queues_sweep_gpu_q$q.json 2>> $O/queues_q$q.err || { tail $O/queues_q$q.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/queues_sweep_gpu_q$q.json')); print('q$q sweep gpu', d['value'], d['ms_per_step'])"
  done
}
step_queues2() {
  # node bench at 4 vs 8 queues (A/B/A/B in one call); 4 blocks per CU (no margin) at 8 queues
  for q in 4 8 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/queues_node_q$q.json 2>> $O/queues2.err || { tail $O/queues2.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/queues_node_q$q.json')); print('q$q node', d['value'], d['ms_per_step'], d.get('gpu_engine',{}).get('insn_share'))"
  done
  ASIM_GPU_BLOCKS_PER_CU=4 timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 > $O/queues_bench_gpu_bpc4.json 2>> $O/queues2.err || { tail $O/queues2.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/queues_bench_gpu_bpc4.json')); print('bpc4 gpu-only', d['value'], d['ms_per_step'])"
  ASIM_GPU_BLOCKS_PER_CU=4 timeout -k 10 400 python3 bench.py --sweep --engine gpu --steps 1 --warmup 0 > $O/queues_sweep_gpu_bpc4.json 2>> $O/queues2.err || { tail $O/queues2.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/queues_sweep_gpu_bpc4.json')); print('bpc4 sweep gpu', d['value'], d['ms_per_step'])"
}
step_chpack() {
  # channels per block of the split build (ASIM_GPU_CH_PER_BLOCK, block_plan in gpu_engine.hip)
  timeout -k 10 600 $PT tests/test_gpu_engine.py -k "split or rodinia_app or snapshot or batch" > $O/pytest_chpack.log 2>&1 || { tail -30 $O/pytest_chpack.log; return 1; }
  tail -2 $O/pytest_chpack.log
  for p in 1 2 4; do
    ASIM_GPU_CH_PER_BLOCK=$p timeout -k 10 240 python3 tools/batch_scaling.py --app hotspot --n 6,8 > $O/chpack_scaling_p$p.jsonl 2> $O/chpack_p$p.err || { tail $O/chpack_p$p.err; return 1; }
    cat $O/chpack_scaling_p$p.jsonl
    ASIM_GPU_CH_PER_BLOCK=$p timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 > $O/chpack_bench_gpu_p$p.json 2>> $O/chpack_p$p.err || { tail $O/chpack_p$p.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/chpack_bench_gpu_p$p.json')); print('p$p gpu-only', d['value'], d['ms_per_step'])"
    ASIM_GPU_CH_PER_BLOCK=$p timeout -k 10 400 python3 bench.py --sweep --engine gpu --steps 1 --warmup 0 > $O/chpack_sweep_gpu_p$p.json 2>> $O/chpack_p$p.err || { tail $O/chpack_p$p.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/chpack_sweep_gpu_p$p.json')); print('p$p sweep gpu', d['value'], d['ms_per_step'])"
  done
}
step_chpack2() {
  # channels per block at the package's default 8 hardware queues (A/B/A/B)
  for p in 1 2 1 2; do
    ASIM_GPU_CH_PER_BLOCK=$p timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 > $O/chpack_q8_bench_gpu_p$p.json 2>> $O/chpack2.err || { tail $O/chpack2.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/chpack_q8_bench_gpu_p$p.json')); print('p$p gpu-only', d['value'], d['ms_per_step'], 'queues', d['gpu_engine'].get('hw_queues'))"
  done
  for p in 1 2; do
    ASIM_GPU_CH_PER_BLOCK=$p timeout -k 10 400 python3 bench.py --sweep --engine gpu --steps 1 --warmup 0 > $O/chpack_q8_sweep_gpu_p$p.json 2>> $O/chpack2.err || { tail $O/chpack2.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/chpack_q8_sweep_gpu_p$p.json')); print('p$p sweep gpu', d['value'], d['ms_per_step'], 'queues', d['gpu_engine'].get('hw_queues'))"
  done
}
step_split2w() {
  # the split build at two waves per SIMD (ASIM_GPU_SPLIT_WAVES=2, engine_k_split2.hip) vs one
  timeout -k 10 120 python3 -c "
import json; from accel_sim_framework_distributed_amd import _native
m = _native.load(); print(json.dumps(m.gpu_engine_modes()))" > $O/engine_modes_split2.json || return 1
  cat $O/engine_modes_split2.json
  ASIM_GPU_SPLIT_WAVES=2 timeout -k 10 600 $PT tests/test_gpu_engine.py -k "split or rodinia_app or snapshot" > $O/pytest_split2w.log 2>&1 || { tail -30 $O/pytest_split2w.log; return 1; }
  tail -2 $O/pytest_split2w.log
  for w in 1 2; do
    ASIM_GPU_SPLIT_WAVES=$w timeout -k 10 120 python3 tools/engine_pmc_1sm.py --app hotspot > $O/one_sm_split_w$w.txt 2>&1 || { tail $O/one_sm_split_w$w.txt; return 1; }
    grep -v amdgpu.ids $O/one_sm_split_w$w.txt | head -3
  done
  for cfg in "1 8" "2 8" "2 16" "1 16"; do
    set -- $cfg
    ASIM_GPU_SPLIT_WAVES=$1 ASIM_GPU_HW_QUEUES=$2 timeout -k 10 300 python3 bench.py --engine gpu --steps 2 --warmup 1 > $O/split2w_bench_gpu_w$1_q$2.json 2>> $O/split2w.err || { tail $O/split2w.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/split2w_bench_gpu_w$1_q$2.json')); print('w$1 q$2 gpu-only', d['value'], d['ms_per_step'], d['gpu_engine'].get('hw_queues'))"
    ASIM_GPU_SPLIT_WAVES=$1 ASIM_GPU_HW_QUEUES=$2 timeout -k 10 400 python3 bench.py --sweep --engine gpu --steps 1 --warmup 0 > $O/split2w_sweep_gpu_w$1_q$2.json 2>> $O/split2w.err || { tail $O/split2w.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/split2w_sweep_gpu_w$1_q$2.json')); print('w$1 q$2 sweep gpu', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'))"
  done
}
step_sweep2w() {
  # node sweep (BASELINE config #5 shape), one vs two engine waves per SIMD, A/B/A/B
  timeout -k 10 300 $PT tests/test_gpu_engine.py -k "kernel_resources" > $O/pytest_resources.log 2>&1 || { tail -30 $O/pytest_resources.log; return 1; }
  tail -2 $O/pytest_resources.log
  for cfg in "1 8" "2 16" "1 8" "2 16"; do
    set -- $cfg
    ASIM_GPU_SPLIT_WAVES=$1 ASIM_GPU_HW_QUEUES=$2 timeout -k 10 400 python3 bench.py --sweep --steps 3 --warmup 1 > $O/sweep2w_node_w$1.json 2>> $O/sweep2w.err || { tail $O/sweep2w.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/sweep2w_node_w$1.json')); print('w$1 q$2 sweep node', d['value'], d['ms_per_step'], d['config'].get('gpu_slots'), d['config'].get('cpu_slots'), d['gpu_engine'])"
    cp $O/sweep2w_node_w$1.json $O/sweep2w_node_w$1_$RANDOM.json
  done
}
step_node2w() {
  # node suite bench (the headline), one vs two engine waves per SIMD, A/B/A/B
  for cfg in "1 8" "2 16" "1 8" "2 16"; do
    set -- $cfg
    ASIM_GPU_SPLIT_WAVES=$1 ASIM_GPU_HW_QUEUES=$2 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/node2w_w$1.json 2>> $O/node2w.err || { tail $O/node2w.err; return 1; }
    python3 -c "import json; d=json.load(open('$O/node2w_w$1.json')); print('w$1 q$2 node', d['value'], d['ms_per_step'], d['gpu_engine'])"
    cp $O/node2w_w$1.json $O/node2w_w$1_$RANDOM.json
  done
}
step_tests() {
  timeout -k 10 1000 $PT tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; return 1; }
  tail -3 $O/pytest_gpu.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; return 1; }
  tail -1 $O/smoke.log
}
step_devloop() {
  # device-resident epoch loop of the packet collective: GPU tests, then the
  # per-epoch cost (host-bounce RCCL, gloo, device loop over RCCL loopback)
  timeout -k 10 300 $PT tests/test_device_exchange.py > $O/pytest_devloop.log 2>&1 || { tail -30 $O/pytest_devloop.log; return 1; }
  tail -3 $O/pytest_devloop.log
  timeout -k 10 300 python3 tools/rccl_epoch_cost.py --iters 1000 --out $O/devloop_epoch_cost.json > $O/devloop_epoch_cost.log 2>&1 \
    || { tail -20 $O/devloop_epoch_cost.log; return 1; }
  grep -v amdgpu.ids $O/devloop_epoch_cost.log | tail -6
}
step_bench() {
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $O/bench_node.json 2> $O/bench_node.err || { tail $O/bench_node.err; return 1; }
  cat $O/bench_node.json
}
for s in "$@"; do
  echo "== $s"
  step_$s || exit 1
done
