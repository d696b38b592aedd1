# One-pass GBM residual kernel: tree tests, then bench A/B at 12.5M and 100M rows.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  tests/test_gpu_algos.py > gpurun_out/pytest_grad.log 2>&1
tail -2 gpurun_out/pytest_grad.log
for R in 12500000 100000000; do
  for G in 0 1; do
    H2O3_GBM_GRAD=$G timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 > gpurun_out/grad_ab.log 2>&1
    echo "rows=$R grad=$G: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/grad_ab.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/grad_ab.log)"
  done
done
