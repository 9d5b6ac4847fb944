set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/profile_engine.py --app bfs > gpurun_out/stage_bfs.log 2>&1
export ASIM_GPU_PROFILE=0
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmc_bfs1 -o pmc -- python3 tools/profile_engine.py --app bfs > gpurun_out/pmc_bfs1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/pmc_bfs2 -o pmc -- python3 tools/profile_engine.py --app bfs > gpurun_out/pmc_bfs2.log 2>&1
