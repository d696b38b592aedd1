#!/bin/bash
# A/B: gram.hip built with and without SLP vectorization (packed f32 VALU
# beside MFMAs): wide Gram kernel, wide GLM iteration, narrow GLM (100M x 100)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r5_slp_ab.txt
: > $o
for arm in base noslp base2; do
  if [ $arm = noslp ]; then
    H2O3_HIPCC_EXTRA=-fno-slp-vectorize timeout -k 10 300 python -c "from h2o3_amd.ops import _native; _native.build_one_hip('gram.hip', force=True)" || exit 1
  fi
  if [ $arm = base2 ]; then
    timeout -k 10 300 python -c "from h2o3_amd.ops import _native; _native.build_one_hip('gram.hip', force=True)" || exit 1
  fi
  echo "== $arm" >> $o
  MB_ARMS=bf16 timeout -k 10 200 python -u scripts/wide_gram_mb.py 2>&1 | grep -v amdgpu.ids >> $o || exit 1
  timeout -k 10 300 python -u bench.py --algo glm --rows 12500000 --cols 1000 --steps 6 --warmup 2 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/wide /' >> $o || exit 1
  timeout -k 10 300 python -u bench.py --algo glm --steps 10 --warmup 3 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/narrow100M /' >> $o || exit 1
  cat $o
done
