set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -n 1 gpurun_out/smoke.log
ONLY=gbm,xgboost,drf,naivebayes,isolationforest H2O3_PROFILE=1 timeout -k 10 600 python -u scripts/algo_survey.py > gpurun_out/algo_survey2.log 2>&1
grep "{" gpurun_out/algo_survey2.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-160
