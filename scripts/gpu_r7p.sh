set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7p
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_devtree_gpu.py tests/test_tree_kernels_gpu.py tests/test_tree_histogram_types.py > gpurun_out/r7p/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7p/tests.log; exit 1; }
tail -1 gpurun_out/r7p/tests.log
timeout -k 10 400 python -u scripts/xgb_automl_prof.py > gpurun_out/r7p/xgb_automl_prof.txt 2>&1 || { echo "xgb prof failed"; tail -20 gpurun_out/r7p/xgb_automl_prof.txt; exit 1; }
head -2 gpurun_out/r7p/xgb_automl_prof.txt
