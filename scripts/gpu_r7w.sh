set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7w
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_linalg_gpu.py -k "wide_tiers" > gpurun_out/r7w/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7w/tests.log; exit 1; }
tail -1 gpurun_out/r7w/tests.log
NFOLDS=0 timeout -k 10 300 python -u scripts/glm_automl_prof.py > gpurun_out/r7w/glm_narrow.txt 2>&1 || { echo "glm narrow failed"; tail -20 gpurun_out/r7w/glm_narrow.txt; exit 1; }
head -2 gpurun_out/r7w/glm_narrow.txt
H2O3_GLM_NARROW_MAX=128 NFOLDS=0 timeout -k 10 300 python -u scripts/glm_automl_prof.py > gpurun_out/r7w/glm_wide.txt 2>&1 || { echo "glm wide failed"; tail -20 gpurun_out/r7w/glm_wide.txt; exit 1; }
head -2 gpurun_out/r7w/glm_wide.txt
