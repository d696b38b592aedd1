#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "tiers or glm" > gpurun_out/r5_tests16.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests16.log; exit 1; fi
tail -2 gpurun_out/r5_tests16.log
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide8.json 2> gpurun_out/r5_glm_wide8.err || { tail -20 gpurun_out/r5_glm_wide8.err; exit 1; }
cat gpurun_out/r5_glm_wide8.json; grep phases gpurun_out/r5_glm_wide8.err
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide9.json 2> gpurun_out/r5_glm_wide9.err || { tail -20 gpurun_out/r5_glm_wide9.err; exit 1; }
cat gpurun_out/r5_glm_wide9.json
timeout -k 10 300 python -u -m pytest tests/test_deeplearning.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_tests16dl.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests16dl.log; exit 1; fi
tail -2 gpurun_out/r5_tests16dl.log
timeout -k 10 300 python -u bench.py --algo dl --rows 10000000 --batch 1024 --steps 400 --warmup 20 \
  > gpurun_out/r5_dl_fused2.json 2> gpurun_out/r5_dl_fused2.err || { tail -20 gpurun_out/r5_dl_fused2.err; exit 1; }
cat gpurun_out/r5_dl_fused2.json
