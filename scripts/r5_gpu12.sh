#!/bin/bash
# round 5: wide GLM tiers (tests + bench with phases), then the full GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "tiers" \
  > gpurun_out/r5_tests12.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests12.log; exit 1; fi
grep -E "passed|failed|FAILED" gpurun_out/r5_tests12.log | tail -5
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 1 \
  > gpurun_out/r5_glm_wide4.json 2> gpurun_out/r5_glm_wide4.err || { tail -20 gpurun_out/r5_glm_wide4.err; exit 1; }
cat gpurun_out/r5_glm_wide4.json; grep phases gpurun_out/r5_glm_wide4.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_pytest_gpu_full.log 2>&1
rc=$?
tail -5 gpurun_out/r5_pytest_gpu_full.log
exit $rc
