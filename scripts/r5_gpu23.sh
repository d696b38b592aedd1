#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests23.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests23.log; exit 1; fi
tail -3 gpurun_out/r5_tests23.log
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide17.json 2> gpurun_out/r5_glm_wide17.err || { tail -20 gpurun_out/r5_glm_wide17.err; exit 1; }
grep phases gpurun_out/r5_glm_wide17.err
for i in 18 19; do
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide$i.json 2> gpurun_out/r5_glm_wide$i.err || { tail -20 gpurun_out/r5_glm_wide$i.err; exit 1; }
cat gpurun_out/r5_glm_wide$i.json
done
