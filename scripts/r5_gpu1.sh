#!/bin/bash
# round 5: GPU numerics (GLM gradient channel, tree bounds), 100M GLM precision, bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_linalg_gpu.py \
  tests/test_tree_kernels_gpu.py tests/test_memory_manager.py > gpurun_out/r5_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r5_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r5_gpu_tests.log
timeout -k 10 500 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
tail -40 gpurun_out/r5_glm_precision.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
