# A/B: write-only leaf scatter + fused add in the residual pass vs in-place RMW leaf update.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  -k "scatter or fill_nid" > gpurun_out/pytest_scatter.log 2>&1 || { tail -30 gpurun_out/pytest_scatter.log; exit 1; }
tail -1 gpurun_out/pytest_scatter.log
for R in 100000000 12500000; do
  for S in 0 1 0 1; do
    H2O3_LEAF_SCATTER=$S timeout -k 10 300 python bench.py --rows $R --steps 20 --warmup 3 --no-glm > gpurun_out/ls.log 2>&1
    echo "rows=$R scatter=$S $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ls.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/ls.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_ls -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-glm > gpurun_out/rocprof_ls.log 2>&1
grep -E "leaf_scatter|leaf_update|gbm_grad" gpurun_out/rocprof_ls/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
rm -f gpurun_out/rocprof_ls/run_kernel_trace.csv
