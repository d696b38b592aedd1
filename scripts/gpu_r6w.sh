set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6w
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_logit_hist_gpu.py > gpurun_out/r6w/tests_lh.log 2>&1 || { echo "lh tests failed"; tail -30 gpurun_out/r6w/tests_lh.log; exit 1; }
tail -1 gpurun_out/r6w/tests_lh.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r6w/tests_all.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/r6w/tests_all.log; exit 1; }
tail -1 gpurun_out/r6w/tests_all.log
timeout -k 10 400 python -u scripts/xgb_automl_prof.py > gpurun_out/r6w/xgb_automl_prof.txt 2>&1 || { echo "xgb prof failed"; tail -20 gpurun_out/r6w/xgb_automl_prof.txt; exit 1; }
head -2 gpurun_out/r6w/xgb_automl_prof.txt
