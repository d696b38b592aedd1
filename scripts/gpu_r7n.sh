set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7n
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_linalg_gpu.py tests/test_coxph_gpu.py tests/test_gpu_algos.py > gpurun_out/r7n/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7n/tests.log; exit 1; }
tail -1 gpurun_out/r7n/tests.log
timeout -k 10 600 python -u scripts/algo_survey2.py > gpurun_out/r7n/algo_survey2.log 2>&1 || { echo "survey2 failed"; tail -20 gpurun_out/r7n/algo_survey2.log; exit 1; }
grep "{" gpurun_out/r7n/algo_survey2.log | cut -c1-120
