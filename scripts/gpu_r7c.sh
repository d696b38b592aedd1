set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7c
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_linalg_gpu.py > gpurun_out/r7c/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7c/tests.log; exit 1; }
tail -2 gpurun_out/r7c/tests.log
timeout -k 10 300 python -u scripts/prof_rulefit.py > gpurun_out/r7c/rulefit_prof.txt 2>&1 || { echo "rulefit prof failed"; tail -20 gpurun_out/r7c/rulefit_prof.txt; exit 1; }
head -3 gpurun_out/r7c/rulefit_prof.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r7c/prof -o rf -- python3 $GRAFT_REPO_ROOT/scripts/prof_rulefit.py > $GRAFT_REPO_ROOT/gpurun_out/r7c/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r7c/rocprof.log; exit 1; }
echo rocprof ok
