#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or tiers" > gpurun_out/r5_tests24.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/r5_tests24.log; exit 1; fi
tail -3 gpurun_out/r5_tests24.log
o=gpurun_out/r5_gram_sw.txt
timeout -k 10 200 python -u scripts/wide_gram_mb.py > $o 2>&1 || { cat $o; exit 1; }
grep -v amdgpu.ids $o
for i in 20 21; do
timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 \
  > gpurun_out/r5_glm_wide$i.json 2> gpurun_out/r5_glm_wide$i.err || { tail -20 gpurun_out/r5_glm_wide$i.err; exit 1; }
cut -c1-200 gpurun_out/r5_glm_wide$i.json
done
