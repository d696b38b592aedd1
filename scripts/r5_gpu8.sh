#!/bin/bash
# round 5: 256-tile fused wide Gram (tests, kernel timings, full pass, wide bench, kernel stats)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "wide" \
  > gpurun_out/r5_tests8.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests8.log; exit 1; fi
grep -E "passed|failed" gpurun_out/r5_tests8.log | tail -3
timeout -k 10 300 python -u scripts/wide_gram_mb.py > gpurun_out/r5_wide_gram_mb2.txt 2>&1 || { tail -20 gpurun_out/r5_wide_gram_mb2.txt; exit 1; }
cat gpurun_out/r5_wide_gram_mb2.txt
timeout -k 10 300 python -u scripts/glm_wide_step_mb.py > gpurun_out/r5_wide_mb2.txt 2>&1 || { tail -20 gpurun_out/r5_wide_mb2.txt; exit 1; }
cat gpurun_out/r5_wide_mb2.txt
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 1 \
  > gpurun_out/r5_glm_wide2.json 2> gpurun_out/r5_glm_wide2.err || { tail -20 gpurun_out/r5_glm_wide2.err; exit 1; }
cat gpurun_out/r5_glm_wide2.json
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_wide3 -o p -- python3 scripts/wide_gram_mb.py 3000000 > gpurun_out/r5_pmc_wide3.log 2>&1 || { tail -20 gpurun_out/r5_pmc_wide3.log; exit 1; }
echo done
