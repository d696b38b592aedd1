set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7j
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_linalg_gpu.py > gpurun_out/r7j/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7j/tests.log; exit 1; }
tail -1 gpurun_out/r7j/tests.log
LDX=711 timeout -k 10 200 python -u scripts/gram_f64_mb.py > gpurun_out/r7j/gram_f64_mb_ld711.txt 2>&1 || { echo "mb failed"; tail -20 gpurun_out/r7j/gram_f64_mb_ld711.txt; exit 1; }
cat gpurun_out/r7j/gram_f64_mb_ld711.txt
