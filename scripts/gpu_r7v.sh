set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7v
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_linalg_gpu.py tests/test_gpu_algos.py tests/test_deeplearning.py > gpurun_out/r7v/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7v/tests.log; exit 1; }
tail -1 gpurun_out/r7v/tests.log
timeout -k 10 400 python -u scripts/glm_automl_prof.py > gpurun_out/r7v/glm_automl_prof.txt 2>&1 || { echo "glm prof failed"; tail -20 gpurun_out/r7v/glm_automl_prof.txt; exit 1; }
head -2 gpurun_out/r7v/glm_automl_prof.txt
