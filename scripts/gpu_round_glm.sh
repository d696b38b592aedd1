# Full GPU test suite + GLM 100M x 100 bench/profile + wide GLM bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --algo glm --steps 20 --warmup 2 > gpurun_out/glm_bench.log 2>&1
tail -n 1 gpurun_out/glm_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_glm100m -o run --output-format csv -- python3 bench.py --algo glm --steps 10 --warmup 2 > gpurun_out/rocprof_glm100m.log 2>&1
rm -f gpurun_out/rocprof_glm100m/run_kernel_trace.csv
timeout -k 10 500 python bench.py --algo glm --rows 12500000 --cols 1000 --steps 5 --warmup 1 > gpurun_out/glm_wide.log 2>&1
grep '"metric"' gpurun_out/glm_wide.log
