#!/bin/bash
# GBM bench A/B on one box: the round-4 tree (ab_r4, git worktree at f94c842) vs HEAD, alternating
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  (cd ab_r4 && timeout -k 10 300 python -u bench.py --no-glm --steps 30 --warmup 3) > gpurun_out/r5_ab_r4_$i.json 2> gpurun_out/r5_ab_r4_$i.err || { tail -20 gpurun_out/r5_ab_r4_$i.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_ab_r4_$i.json
  timeout -k 10 300 python -u bench.py --no-glm --steps 30 --warmup 3 > gpurun_out/r5_ab_head_$i.json 2> gpurun_out/r5_ab_head_$i.err || { tail -20 gpurun_out/r5_ab_head_$i.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5_ab_head_$i.json
done
