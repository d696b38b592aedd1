#!/bin/bash
# round 5: fused DL MLP step (tests, bench fused vs unfused, rocprof), then the
# GLM gradient-channel cost, 100M precision, the flagship bench and a GLM profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_deeplearning.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r5_dl_tests.log 2>&1 || { tail -40 gpurun_out/r5_dl_tests.log; exit 1; }
tail -3 gpurun_out/r5_dl_tests.log
timeout -k 10 300 python -u bench.py --algo dl --rows 10000000 --batch 1024 --steps 400 --warmup 20 \
  > gpurun_out/r5_dl_fused.json 2> gpurun_out/r5_dl_fused.err || { tail -20 gpurun_out/r5_dl_fused.err; exit 1; }
cat gpurun_out/r5_dl_fused.json
H2O3_DL_FUSED=0 timeout -k 10 300 python -u bench.py --algo dl --rows 10000000 --batch 1024 --steps 400 --warmup 20 \
  > gpurun_out/r5_dl_unfused.json 2> gpurun_out/r5_dl_unfused.err || { tail -20 gpurun_out/r5_dl_unfused.err; exit 1; }
cat gpurun_out/r5_dl_unfused.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl_r5 -o dl --output-format csv -- python3 bench.py --algo dl --rows 10000000 --batch 1024 --steps 200 --warmup 10 \
  > gpurun_out/r5_prof_dl.log 2>&1 || { tail -20 gpurun_out/r5_prof_dl.log; exit 1; }
find gpurun_out/prof_dl_r5 -name "*kernel_stats.csv"
for g in 0 1 2; do
  H2O3_MB_GRAD=$g timeout -k 10 200 python -u scripts/glm_ws_mb.py >> gpurun_out/r5_glm_ws_mb.txt 2>&1 || { tail -20 gpurun_out/r5_glm_ws_mb.txt; exit 1; }
done
cat gpurun_out/r5_glm_ws_mb.txt
timeout -k 10 600 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
cat gpurun_out/glm_precision_100m_r5.json
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_glm_r5 -o glm --output-format csv -- python3 bench.py --algo glm --steps 10 --warmup 3 \
  > gpurun_out/r5_prof_glm.log 2>&1 || { tail -20 gpurun_out/r5_prof_glm.log; exit 1; }
find gpurun_out/prof_glm_r5 -name "*kernel_stats.csv"
