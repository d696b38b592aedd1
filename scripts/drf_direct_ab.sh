# Row-direct pair histograms for column-sampled levels: kernel tests, then the
# DRF config (10M x 500, 100 categoricals of cardinality 1000) with the direct
# path at every sampled level / node-batched levels only (auto) / off.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  > gpurun_out/pytest_pairs.log 2>&1
tail -3 gpurun_out/pytest_pairs.log
for D in ${DLIST:-1 auto 0}; do
  H2O3_PAIR_DIRECT=$D H2O3_PROFILE=1 timeout -k 10 400 python bench.py --algo drf --rows 10000000 --cols 500 \
    --cat-cols 100 --cat-card 1000 --steps 3 --warmup 1 > gpurun_out/drf_direct_$D.log 2>&1
  echo "direct=$D"; grep '"metric"' gpurun_out/drf_direct_$D.log | cut -c1-300
done
H2O3_PAIR_DIRECT=1 BENCH_ARGS="--algo drf --rows 10000000 --cols 500 --cat-cols 100 --cat-card 1000 --steps 2 --warmup 1" \
  timeout -k 10 400 python scripts/grow_line_sampler.py > gpurun_out/drf_lines.txt 2>&1
