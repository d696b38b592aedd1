set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7h
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_linalg_gpu.py > gpurun_out/r7h/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r7h/tests.log; exit 1; }
tail -2 gpurun_out/r7h/tests.log
timeout -k 10 200 python -u scripts/gram_f64_mb.py > gpurun_out/r7h/gram_f64_mb.txt 2>&1 || { echo "mb failed"; tail -20 gpurun_out/r7h/gram_f64_mb.txt; exit 1; }
cat gpurun_out/r7h/gram_f64_mb.txt
timeout -k 10 300 python -u scripts/prof_rulefit.py > gpurun_out/r7h/rulefit_prof.txt 2>&1 || { echo "rulefit prof failed"; tail -20 gpurun_out/r7h/rulefit_prof.txt; exit 1; }
head -3 gpurun_out/r7h/rulefit_prof.txt
