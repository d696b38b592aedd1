# Tiled fill_nid: GPU tree tests + default DRF timing (2M x 50) + DRF 10M x 500 bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  tests/test_gpu_algos.py > gpurun_out/pytest_nid.log 2>&1 || { tail -30 gpurun_out/pytest_nid.log; exit 1; }
tail -2 gpurun_out/pytest_nid.log
timeout -k 10 300 python -u scripts/drf_default_timing.py > gpurun_out/drf_default.log 2>&1
cat gpurun_out/drf_default.log | grep -v amdgpu.ids
timeout -k 10 400 python bench.py --algo drf --rows 10000000 --cols 500 --cat-cols 100 --cat-card 1000 --steps 3 \
  --warmup 1 > gpurun_out/nid_drf.log 2>&1
echo "drf 10Mx500: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nid_drf.log)"
