# GLM 100M x 100 bench + rocprofv3 kernel stats (bf16x3 MFMA default).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glm.log 2>&1 || { tail -30 gpurun_out/pytest_glm.log; exit 1; }
tail -n 1 gpurun_out/pytest_glm.log
timeout -k 10 300 python bench.py --algo glm --steps 20 --warmup 2 > gpurun_out/glm_bench.log 2>&1
tail -n 1 gpurun_out/glm_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_glm100m -o run --output-format csv -- python3 bench.py --algo glm --steps 10 --warmup 2 > gpurun_out/rocprof_glm100m.log 2>&1
head -6 gpurun_out/rocprof_glm100m/run_kernel_stats.csv | cut -c1-220
