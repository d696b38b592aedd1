#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests21.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests21.log; exit 1; fi
tail -2 gpurun_out/r5_tests21.log
o=gpurun_out/r5_eta_mb2.txt
timeout -k 10 200 python -u scripts/wide_eta_mb.py 0 1024 1536 2048 3072 > $o 2>&1 || { cat $o; exit 1; }
grep -v amdgpu.ids $o
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide14.json 2> gpurun_out/r5_glm_wide14.err || { tail -20 gpurun_out/r5_glm_wide14.err; exit 1; }
grep phases gpurun_out/r5_glm_wide14.err
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide15.json 2> gpurun_out/r5_glm_wide15.err || { tail -20 gpurun_out/r5_glm_wide15.err; exit 1; }
cat gpurun_out/r5_glm_wide15.json
