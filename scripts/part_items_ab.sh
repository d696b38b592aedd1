set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  > gpurun_out/pytest_items.log 2>&1
tail -2 gpurun_out/pytest_items.log
for R in 12500000 100000000; do
  for I in host dev; do
    H2O3_PART_ITEMS=$I timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 > gpurun_out/items_ab.log 2>&1
    echo "rows=$R items=$I: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/items_ab.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/items_ab.log)"
  done
done
