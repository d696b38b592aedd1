#!/bin/bash
# round 5: wide GLM after the assembly fix (tests, bench with phases), flagship bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests15.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests15.log; exit 1; fi
tail -2 gpurun_out/r5_tests15.log
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide7.json 2> gpurun_out/r5_glm_wide7.err || { tail -20 gpurun_out/r5_glm_wide7.err; exit 1; }
cat gpurun_out/r5_glm_wide7.json; grep phases gpurun_out/r5_glm_wide7.err
H2O3_GLM_WIDE_FUSED=0 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide_split.json 2> gpurun_out/r5_glm_wide_split.err || { tail -20 gpurun_out/r5_glm_wide_split.err; exit 1; }
cat gpurun_out/r5_glm_wide_split.json
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench2.json 2> gpurun_out/r5_bench2.err || { tail -20 gpurun_out/r5_bench2.err; exit 1; }
cat gpurun_out/r5_bench2.json
