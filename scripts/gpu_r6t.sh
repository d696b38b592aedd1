set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6t
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_devtree_gpu.py tests/test_tree_histogram_types.py tests/test_ua_fold_gpu.py tests/test_tree_kernels_gpu.py > gpurun_out/r6t/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6t/tests.log; exit 1; }
tail -1 gpurun_out/r6t/tests.log
timeout -k 10 400 python -u scripts/gbm_automl_prof.py > gpurun_out/r6t/gbm_automl_prof.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6t/gbm_automl_prof.txt; exit 1; }
head -2 gpurun_out/r6t/gbm_automl_prof.txt
timeout -k 10 400 python -u scripts/xgb_automl_prof.py > gpurun_out/r6t/xgb_automl_prof.txt 2>&1 || { echo "xgb prof failed"; tail -20 gpurun_out/r6t/xgb_automl_prof.txt; exit 1; }
head -2 gpurun_out/r6t/xgb_automl_prof.txt
