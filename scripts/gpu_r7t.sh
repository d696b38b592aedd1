set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7t
timeout -k 10 450 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_distributed_gpu.py > gpurun_out/r7t/tests.log 2>&1 || { echo "dist test failed"; exit 1; }
tail -2 gpurun_out/r7t/tests.log
