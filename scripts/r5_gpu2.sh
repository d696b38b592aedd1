#!/bin/bash
# round 5: GLM precision at 100M (three Hessian modes vs fp64), bench, GLM kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_memory_manager.py \
  > gpurun_out/r5_mem.log 2>&1 || { tail -30 gpurun_out/r5_mem.log; exit 1; }
tail -2 gpurun_out/r5_mem.log
timeout -k 10 600 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
tail -40 gpurun_out/r5_glm_precision.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_glm_r5 -o glm -- python3 bench.py --algo glm --steps 10 --warmup 3 \
  > gpurun_out/r5_prof_glm.log 2>&1 || { tail -20 gpurun_out/r5_prof_glm.log; exit 1; }
find gpurun_out/prof_glm_r5 -name "*kernel_stats.csv" | head -3
