set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6r
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests -k "gbm or devtree or tree or forest" > gpurun_out/r6r/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6r/tests.log; exit 1; }
tail -1 gpurun_out/r6r/tests.log
H2O3_PROFILE=0 timeout -k 10 400 python -u scripts/gbm_automl_prof.py > gpurun_out/r6r/gbm_automl_prof.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6r/gbm_automl_prof.txt; exit 1; }
head -4 gpurun_out/r6r/gbm_automl_prof.txt
H2O3_PROFILE=0 timeout -k 10 400 python -u scripts/xgb_automl_prof.py > gpurun_out/r6r/xgb_automl_prof.txt 2>&1 || { echo "xgb prof failed"; tail -20 gpurun_out/r6r/xgb_automl_prof.txt; exit 1; }
head -4 gpurun_out/r6r/xgb_automl_prof.txt
