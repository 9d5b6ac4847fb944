#!/bin/bash
# concurrency check of the cross-process CU reservation, then the correlation pipeline
set -e
timeout -k 10 200 bash tools/repro/conc.sh
bash tools/gpu_correlate.sh
