# Host-overhead diet: tree GPU tests, host floor, bench at 12.5M and 100M.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_kernels_gpu.py tests/test_gbm.py tests/test_trees_more.py -m gpu > gpurun_out/pytest_diet.log 2>&1 || { tail -40 gpurun_out/pytest_diet.log; exit 1; }
tail -n 1 gpurun_out/pytest_diet.log
timeout -k 10 300 python scripts/host_floor.py > gpurun_out/host_floor2.txt 2>&1
head -30 gpurun_out/host_floor2.txt | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --rows 12500000 --steps 20 --warmup 3 --no-glm > gpurun_out/diet_12m5.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/diet_12m5.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-glm > gpurun_out/diet_100m.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/diet_100m.log
