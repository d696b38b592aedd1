# Bin-major conflict-free histogram kernel: GPU tests, then GBM A/B vs the grouped-lane kernel.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_kernels_gpu.py -m gpu > gpurun_out/pytest_bm.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/pytest_bm.log; exit 1; }
tail -n 3 gpurun_out/pytest_bm.log
for R in 100000000 12500000; do
  for BM in 1 0; do
    H2O3_HIST_BM=$BM timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 --no-glm > gpurun_out/bm_${BM}_$R.log 2>&1
    echo "rows=$R bm=$BM $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bm_${BM}_$R.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/bm_${BM}_$R.log)"
  done
done
