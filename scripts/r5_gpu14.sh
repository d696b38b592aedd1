#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/cond_timing.py > gpurun_out/r5_cond_timing.txt 2>&1 || { tail -20 gpurun_out/r5_cond_timing.txt; exit 1; }
cat gpurun_out/r5_cond_timing.txt
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 1 \
  > gpurun_out/r5_glm_wide6.json 2> gpurun_out/r5_glm_wide6.err || { tail -20 gpurun_out/r5_glm_wide6.err; exit 1; }
cat gpurun_out/r5_glm_wide6.json; grep phases gpurun_out/r5_glm_wide6.err
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests14.log 2>&1
tail -2 gpurun_out/r5_tests14.log
