set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6s
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_devtree_gpu.py > gpurun_out/r6s/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6s/tests.log; exit 1; }
tail -1 gpurun_out/r6s/tests.log
timeout -k 10 400 python -u scripts/gbm_automl_prof.py > gpurun_out/r6s/gbm_automl_prof.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6s/gbm_automl_prof.txt; exit 1; }
head -2 gpurun_out/r6s/gbm_automl_prof.txt
timeout -k 10 400 python -u scripts/xgb_automl_prof.py > gpurun_out/r6s/xgb_automl_prof.txt 2>&1 || { echo "xgb prof failed"; tail -20 gpurun_out/r6s/xgb_automl_prof.txt; exit 1; }
head -2 gpurun_out/r6s/xgb_automl_prof.txt
