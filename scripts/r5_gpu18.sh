#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests18.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests18.log; exit 1; fi
tail -2 gpurun_out/r5_tests18.log
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide10.json 2> gpurun_out/r5_glm_wide10.err || { tail -20 gpurun_out/r5_glm_wide10.err; exit 1; }
cat gpurun_out/r5_glm_wide10.json; grep phases gpurun_out/r5_glm_wide10.err
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide11.json 2> gpurun_out/r5_glm_wide11.err || { tail -20 gpurun_out/r5_glm_wide11.err; exit 1; }
cat gpurun_out/r5_glm_wide11.json
H2O3_GLM_DEV_SOLVE=0 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide12.json 2> gpurun_out/r5_glm_wide12.err || { tail -20 gpurun_out/r5_glm_wide12.err; exit 1; }
cat gpurun_out/r5_glm_wide12.json
