# Round-2 end check: GPU tests, smoke, default bench (GBM + GLM), GLM lambda-search phases.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -n 2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log
H2O3_PROFILE=1 timeout -k 10 300 python scripts/glm_lambda_search.py 12500000 1000 30 > gpurun_out/glm_ls.log 2>&1
tail -2 gpurun_out/glm_ls.log
