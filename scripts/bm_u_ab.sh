# bm kernel load depth A/B (U = 4 vs 8 rows per lane per iteration) at 100M and 12.5M rows.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_kernels_gpu.py -m gpu -k "bm" > gpurun_out/pytest_bmu.log 2>&1 || { tail -40 gpurun_out/pytest_bmu.log; exit 1; }
H2O3_HIST_BM_LW=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_kernels_gpu.py -m gpu -k "bm" >> gpurun_out/pytest_bmu.log 2>&1 || { tail -40 gpurun_out/pytest_bmu.log; exit 1; }
tail -n 2 gpurun_out/pytest_bmu.log
for R in 100000000 12500000; do
  for U in 2 1; do
    H2O3_HIST_BM_LW=$U timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 --no-glm > gpurun_out/bmu_${U}_$R.log 2>&1
    echo "rows=$R LW=$U $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bmu_${U}_$R.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/bmu_${U}_$R.log)"
  done
done
