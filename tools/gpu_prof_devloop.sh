set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/devprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/devprof -o run -- python3 tools/rccl_epoch_cost.py --iters 200 > gpurun_out/devprof/log.txt 2>&1 || { tail -20 gpurun_out/devprof/log.txt; exit 1; }
find gpurun_out/devprof -name "*kernel_stats.csv" | head -3
for f in $(find gpurun_out/devprof -name "*kernel_stats.csv"); do head -12 $f | cut -c1-250; done
