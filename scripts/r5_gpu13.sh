#!/bin/bash
# round 5: where the wide GLM iteration goes (phases + kernel stats)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
H2O3_PROFILE=1 timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 1 \
  > gpurun_out/r5_glm_wide5.json 2> gpurun_out/r5_glm_wide5.err || { tail -20 gpurun_out/r5_glm_wide5.err; exit 1; }
cat gpurun_out/r5_glm_wide5.json; grep phases gpurun_out/r5_glm_wide5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wide_r5b -o wide --output-format csv -- python3 bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 1 \
  > gpurun_out/r5_prof_wide_b.log 2>&1 || { tail -20 gpurun_out/r5_prof_wide_b.log; exit 1; }
find gpurun_out/prof_wide_r5b -name "*_trace.csv" -delete
head -12 gpurun_out/prof_wide_r5b/wide_kernel_stats.csv | cut -c1-160
