# GLM bf16x3 kernel with the swizzled LDS image: GPU tests + bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_linalg_gpu.py tests/test_glm.py -m gpu > gpurun_out/pytest_glm.log 2>&1 || { tail -40 gpurun_out/pytest_glm.log; exit 1; }
tail -n 2 gpurun_out/pytest_glm.log
timeout -k 10 300 python bench.py --algo glm --steps 20 --warmup 3 > gpurun_out/glm_swz.log 2>&1
grep -o '"ms_per_step": [0-9.]*\|"train_deviance_per_row": [0-9.]*' gpurun_out/glm_swz.log
timeout -k 10 300 python bench.py --algo glm --rows 12500000 --steps 20 --warmup 3 > gpurun_out/glm_swz_12m5.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/glm_swz_12m5.log
