#!/bin/bash
# round 5: wide GLM with the bf16 Hessian tier (tier tests, bench with phases), DRF W=8 bytes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "wide or tiers" \
  > gpurun_out/r5_tests11.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests11.log; exit 1; fi
grep -E "passed|failed|FAILED" gpurun_out/r5_tests11.log | tail -5
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 1 \
  > gpurun_out/r5_glm_wide3.json 2> gpurun_out/r5_glm_wide3.err || { tail -20 gpurun_out/r5_glm_wide3.err; exit 1; }
cat gpurun_out/r5_glm_wide3.json; grep phases gpurun_out/r5_glm_wide3.err
bash scripts/r5_coll_drf.sh
