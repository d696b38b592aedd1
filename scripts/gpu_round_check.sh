# GPU tests + smoke + GBM/GLM default benches (one gpurun call).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -n 2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-400
timeout -k 10 400 python bench.py --algo glm > gpurun_out/bench_glm.log 2>&1
tail -1 gpurun_out/bench_glm.log | cut -c1-400
