# Partition compaction A/B (stride count per iteration, work-item size) at the
# per-GPU share of the 100M config at 8 GPUs and at 100M rows.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  -k "partition or grow_async or lookahead or position_leaf" > gpurun_out/pytest_part.log 2>&1
tail -2 gpurun_out/pytest_part.log
for R in 12500000 100000000; do
  for CFG in "H2O3_PART_U=1 H2O3_PART_CHUNK=16384" "H2O3_PART_U=4 H2O3_PART_CHUNK=16384" "H2O3_PART_U=4"; do
    env $CFG timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 > gpurun_out/part_ab.log 2>&1
    echo "rows=$R $CFG: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/part_ab.log)"
  done
done
