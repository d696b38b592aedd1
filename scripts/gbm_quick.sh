set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tree_kernels_gpu.py tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1 || { tail -40 gpurun_out/pytest_tree.log; exit 1; }
tail -n 1 gpurun_out/pytest_tree.log
for R in 12500000 100000000; do
  timeout -k 10 300 python bench.py --rows $R --steps 20 --warmup 3 > gpurun_out/gbm_$R.log 2>&1
  echo "rows=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gbm_$R.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/gbm_$R.log)"
done
