#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests19.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests19.log; exit 1; fi
tail -2 gpurun_out/r5_tests19.log
for rw in 1 2 4; do
H2O3_WIDE_RW=$rw H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_rw$rw.json 2> gpurun_out/r5_glm_rw$rw.err || { tail -20 gpurun_out/r5_glm_rw$rw.err; exit 1; }
echo "RW=$rw"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_glm_rw$rw.json; grep -o "'glm.wide_eta': ([0-9.]*" gpurun_out/r5_glm_rw$rw.err
done
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide13.json 2> gpurun_out/r5_glm_wide13.err || { tail -20 gpurun_out/r5_glm_wide13.err; exit 1; }
cat gpurun_out/r5_glm_wide13.json
