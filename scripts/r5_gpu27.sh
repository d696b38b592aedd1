#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_tests27.log 2>&1
rc=$?
tail -3 gpurun_out/r5_tests27.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r5_tests27.log | head -20; exit 1; fi
timeout -k 10 300 python -u bench.py --algo glm --steps 10 --warmup 3 > gpurun_out/r5_glm_narrow_bf16.json 2> gpurun_out/r5_glm_narrow_bf16.err || { tail -20 gpurun_out/r5_glm_narrow_bf16.err; exit 1; }
cut -c1-220 gpurun_out/r5_glm_narrow_bf16.json
grep -o '"iters": [0-9]*, "hessian_tier": "[a-z0-9]*", "hessian_kappa": [0-9.]*' gpurun_out/r5_glm_narrow_bf16.json
timeout -k 10 600 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_bf16_r5.json > gpurun_out/r5_prec.log 2>&1 || { tail -20 gpurun_out/r5_prec.log; exit 1; }
tail -45 gpurun_out/r5_prec.log
