#!/bin/bash
# round 5: GLM exact-gradient channel -- GPU numerics tests, 100M precision run, bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_linalg_gpu.py \
  > gpurun_out/r5_linalg_gpu.log 2>&1 || { tail -50 gpurun_out/r5_linalg_gpu.log; exit 1; }
tail -3 gpurun_out/r5_linalg_gpu.log
timeout -k 10 500 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
tail -40 gpurun_out/r5_glm_precision.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
