set -e
export TMPDIR=/tmp
timeout -k 10 200 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
H2O3_PROFILE=1 timeout -k 10 200 python bench.py --rows 10000000 --steps 3 --warmup 1 > gpurun_out/qb10m.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/qb10m.log; grep phases gpurun_out/qb10m.log | cut -c1-300
H2O3_PROFILE=1 timeout -k 10 400 python bench.py --rows 100000000 --steps 3 --warmup 1 > gpurun_out/qb100m.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/qb100m.log; grep phases gpurun_out/qb100m.log | cut -c1-300
