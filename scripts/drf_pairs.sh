set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tree_kernels_gpu.py tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1 || { tail -40 gpurun_out/pytest_tree.log; exit 1; }
tail -n 1 gpurun_out/pytest_tree.log
H2O3_PROFILE=1 timeout -k 10 400 python bench.py --algo drf --rows ${ROWS:-10000000} --cols 500 --cat-cols 100 --cat-card 1000 \
  --steps 5 --warmup 1 > gpurun_out/drf_bench.log 2>&1
grep '"metric"' gpurun_out/drf_bench.log | cut -c1-300
grep phases gpurun_out/drf_bench.log | cut -c1-400 || true
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/gbm_bench.log 2>&1
tail -n 1 gpurun_out/gbm_bench.log | cut -c1-250
