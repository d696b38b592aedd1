set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7m
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_coxph_gpu.py > gpurun_out/r7m/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7m/tests.log; exit 1; }
tail -2 gpurun_out/r7m/tests.log
for a in coxph isolationforest extendedisolationforest; do
  ALGO=$a timeout -k 10 300 python -u scripts/prof_any.py > gpurun_out/r7m/prof_$a.txt 2>&1 || { echo "$a prof failed"; tail -20 gpurun_out/r7m/prof_$a.txt; exit 1; }
  grep train_s gpurun_out/r7m/prof_$a.txt
done
