set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_devtree_gpu.py > gpurun_out/r6y/tests_dt.log 2>&1 || { echo "devtree tests failed"; tail -40 gpurun_out/r6y/tests_dt.log; exit 1; }
tail -3 gpurun_out/r6y/tests_dt.log
