# Two-pass histogram flush: GPU tests (bm + tree kernels), microbenchmark, GBM A/B.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_kernels_gpu.py -m gpu > gpurun_out/pytest_red.log 2>&1 || { tail -40 gpurun_out/pytest_red.log; exit 1; }
tail -n 2 gpurun_out/pytest_red.log
timeout -k 10 300 python scripts/hist_bm_mb.py > gpurun_out/hist_bm_mb_red.txt 2>&1
cat gpurun_out/hist_bm_mb_red.txt
for R in 100000000 12500000; do
  for RED in 1 0; do
    H2O3_HIST_BM_RED=$RED timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 --no-glm > gpurun_out/red_${RED}_$R.log 2>&1
    echo "rows=$R red=$RED $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/red_${RED}_$R.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/red_${RED}_$R.log)"
  done
done
