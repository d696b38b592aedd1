#!/bin/bash
# round 5: fused DL step + fused wide Gram after the latency fixes (tests,
# microbench, benches, kernel stats), partition-free histogram microbench,
# GLM narrow gradient-channel cost + 100M precision + flagship bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
prof_clean() { find "$1" -name "*_trace.csv" -delete; find "$1" -name "*.db" -delete; true; }
timeout -k 10 300 python -u -m pytest tests/test_deeplearning.py tests/test_linalg_gpu.py tests/test_tree_kernels_gpu.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "dl_ or wide or pair_narrow" > gpurun_out/r5_tests6.log 2>&1
rc=$?
# an assertion failure (rc 1) is read afterwards; anything else (fault, abort, time limit) ends the run
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests6.log; exit 1; fi
grep -E "passed|failed" gpurun_out/r5_tests6.log | tail -1
timeout -k 10 300 python -u scripts/glm_wide_step_mb.py > gpurun_out/r5_wide_mb.txt 2>&1 || { tail -20 gpurun_out/r5_wide_mb.txt; exit 1; }
cat gpurun_out/r5_wide_mb.txt
timeout -k 10 300 python -u bench.py --algo dl --rows 10000000 --batch 1024 --steps 400 --warmup 20 \
  > gpurun_out/r5_dl_fused.json 2> gpurun_out/r5_dl_fused.err || { tail -20 gpurun_out/r5_dl_fused.err; exit 1; }
cat gpurun_out/r5_dl_fused.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl_r5 -o dl --output-format csv -- python3 bench.py --algo dl --rows 10000000 --batch 1024 --steps 200 --warmup 10 \
  > gpurun_out/r5_prof_dl.log 2>&1 || { tail -20 gpurun_out/r5_prof_dl.log; exit 1; }
prof_clean gpurun_out/prof_dl_r5
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 3 --warmup 1 \
  > gpurun_out/r5_glm_wide.json 2> gpurun_out/r5_glm_wide.err || { tail -20 gpurun_out/r5_glm_wide.err; exit 1; }
cat gpurun_out/r5_glm_wide.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wide_r5 -o wide --output-format csv -- python3 bench.py --algo glm --rows 12500000 --cols 1000 --steps 3 --warmup 1 \
  > gpurun_out/r5_prof_wide.log 2>&1 || { tail -20 gpurun_out/r5_prof_wide.log; exit 1; }
prof_clean gpurun_out/prof_wide_r5
timeout -k 10 120 ./scripts/pf_hist_mb 12500000 > gpurun_out/r5_pf_hist_12m5.json 2>&1 || { tail -20 gpurun_out/r5_pf_hist_12m5.json; exit 1; }
cat gpurun_out/r5_pf_hist_12m5.json
for g in 0 1 2; do
  H2O3_MB_GRAD=$g timeout -k 10 200 python -u scripts/glm_ws_mb.py >> gpurun_out/r5_glm_ws_mb.txt 2>&1 || { tail -20 gpurun_out/r5_glm_ws_mb.txt; exit 1; }
done
cat gpurun_out/r5_glm_ws_mb.txt
timeout -k 10 600 python -u scripts/glm_precision.py --out gpurun_out/glm_precision_100m_r5.json \
  > gpurun_out/r5_glm_precision.log 2>&1 || { tail -30 gpurun_out/r5_glm_precision.log; exit 1; }
cat gpurun_out/glm_precision_100m_r5.json
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
