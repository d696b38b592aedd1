set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7e
timeout -k 10 450 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_distributed_gpu.py > gpurun_out/r7e/tests.log 2>&1 || { echo "dist test failed"; tail -60 gpurun_out/r7e/tests.log; exit 1; }
tail -2 gpurun_out/r7e/tests.log
timeout -k 10 700 python -u scripts/munging_survey.py > gpurun_out/r7e/munging_survey.log 2>&1 || { echo "munging survey failed"; tail -20 gpurun_out/r7e/munging_survey.log; exit 1; }
grep "{" gpurun_out/r7e/munging_survey.log | cut -c1-150
