# Vectorized level bookkeeping: GPU tree tests, GBM bench at 12.5M / 100M,
# DRF (default params on 2M x 50; the 10M x 500 mixed config).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  tests/test_gpu_algos.py > gpurun_out/pytest_vec.log 2>&1
tail -2 gpurun_out/pytest_vec.log
for R in 12500000 100000000; do
  timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 > gpurun_out/vec_gbm.log 2>&1
  echo "gbm rows=$R: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vec_gbm.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/vec_gbm.log)"
done
timeout -k 10 300 python -u scripts/drf_default_timing.py > gpurun_out/drf_default.log 2>&1
grep ntrees gpurun_out/drf_default.log
timeout -k 10 400 python bench.py --algo drf --rows 10000000 --cols 500 --cat-cols 100 --cat-card 1000 --steps 3 \
  --warmup 1 > gpurun_out/vec_drf.log 2>&1
echo "drf 10Mx500: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vec_drf.log)"
