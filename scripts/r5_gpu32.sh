#!/bin/bash
# rocprofv3 kernel stats: wide GLM (12.5M x 1000) and narrow GLM (100M x 100, bf16 tier)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_glm_wide -o run --output-format csv -- python3 bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 > gpurun_out/prof_glm_wide.log 2>&1 || { tail -20 gpurun_out/prof_glm_wide.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_glm_narrow -o run --output-format csv -- python3 bench.py --algo glm --steps 10 --warmup 3 > gpurun_out/prof_glm_narrow.log 2>&1 || { tail -20 gpurun_out/prof_glm_narrow.log; exit 1; }
find gpurun_out/prof_glm_wide gpurun_out/prof_glm_narrow -name "*kernel_trace.csv" -delete
find gpurun_out/prof_glm_wide gpurun_out/prof_glm_narrow -name "*kernel_stats.csv" | head
grep -h ms_per_step gpurun_out/prof_glm_wide.log gpurun_out/prof_glm_narrow.log | cut -c1-200
