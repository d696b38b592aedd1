#!/bin/bash
# round 5: GLM gradient-channel cost (kernel microbench), precision at 100M, bench, GLM profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 0 1 2; do
  H2O3_MB_GRAD=$g timeout -k 10 200 python -u scripts/glm_ws_mb.py >> gpurun_out/r5_glm_ws_mb.txt 2>&1 || { tail -20 gpurun_out/r5_glm_ws_mb.txt; exit 1; }
done
cat gpurun_out/r5_glm_ws_mb.txt | grep ms/pass
timeout -k 10 600 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
cat gpurun_out/glm_precision_100m_r5.json
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_glm_r5 -o glm -- python3 bench.py --algo glm --steps 10 --warmup 3 \
  > gpurun_out/r5_prof_glm.log 2>&1 || { tail -20 gpurun_out/r5_prof_glm.log; exit 1; }
find gpurun_out/prof_glm_r5 -name "*kernel_stats.csv"
