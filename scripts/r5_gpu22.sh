#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests22.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests22.log; exit 1; fi
tail -3 gpurun_out/r5_tests22.log
o=gpurun_out/r5_gram_kr.txt
H2O3_WIDE_KR=32 MB_ARMS=bf16 timeout -k 10 200 python -u scripts/wide_gram_mb.py > $o 2>&1 || { cat $o; exit 1; }
MB_ARMS=bf16 timeout -k 10 200 python -u scripts/wide_gram_mb.py >> $o 2>&1 || { cat $o; exit 1; }
grep -v amdgpu.ids $o
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide16.json 2> gpurun_out/r5_glm_wide16.err || { tail -20 gpurun_out/r5_glm_wide16.err; exit 1; }
cat gpurun_out/r5_glm_wide16.json
