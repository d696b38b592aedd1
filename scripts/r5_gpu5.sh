#!/bin/bash
# round 5: fused DL step + fused wide Gram (tests, microbench), DL bench A/B,
# wide GLM bench, rocprof; then the GLM narrow precision + flagship bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_deeplearning.py tests/test_linalg_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "dl_ or wide" > gpurun_out/r5_tests5.log 2>&1 || { tail -40 gpurun_out/r5_tests5.log; exit 1; }
grep -c PASSED gpurun_out/r5_tests5.log
timeout -k 10 300 python -u scripts/glm_wide_step_mb.py > gpurun_out/r5_wide_mb.txt 2>&1 || { tail -20 gpurun_out/r5_wide_mb.txt; exit 1; }
cat gpurun_out/r5_wide_mb.txt
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 3 --warmup 1 \
  > gpurun_out/r5_glm_wide.json 2> gpurun_out/r5_glm_wide.err || { tail -20 gpurun_out/r5_glm_wide.err; exit 1; }
cat gpurun_out/r5_glm_wide.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wide_r5 -o wide --output-format csv -- python3 bench.py --algo glm --rows 12500000 --cols 1000 --steps 3 --warmup 1 \
  > gpurun_out/r5_prof_wide.log 2>&1 || { tail -20 gpurun_out/r5_prof_wide.log; exit 1; }
timeout -k 10 300 python -u bench.py --algo dl --rows 10000000 --batch 1024 --steps 400 --warmup 20 \
  > gpurun_out/r5_dl_fused.json 2> gpurun_out/r5_dl_fused.err || { tail -20 gpurun_out/r5_dl_fused.err; exit 1; }
cat gpurun_out/r5_dl_fused.json
H2O3_DL_FUSED=0 timeout -k 10 300 python -u bench.py --algo dl --rows 10000000 --batch 1024 --steps 400 --warmup 20 \
  > gpurun_out/r5_dl_unfused.json 2> gpurun_out/r5_dl_unfused.err || { tail -20 gpurun_out/r5_dl_unfused.err; exit 1; }
cat gpurun_out/r5_dl_unfused.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl_r5 -o dl --output-format csv -- python3 bench.py --algo dl --rows 10000000 --batch 1024 --steps 200 --warmup 10 \
  > gpurun_out/r5_prof_dl.log 2>&1 || { tail -20 gpurun_out/r5_prof_dl.log; exit 1; }
for g in 0 1 2; do
  H2O3_MB_GRAD=$g timeout -k 10 200 python -u scripts/glm_ws_mb.py >> gpurun_out/r5_glm_ws_mb.txt 2>&1 || { tail -20 gpurun_out/r5_glm_ws_mb.txt; exit 1; }
done
cat gpurun_out/r5_glm_ws_mb.txt
timeout -k 10 600 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
cat gpurun_out/glm_precision_100m_r5.json
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
