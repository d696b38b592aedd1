set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6k
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_devtree_gpu.py > gpurun_out/r6k/tests.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAIL" gpurun_out/r6k/tests.log | head -30; exit 1; }
echo "tests ok"
