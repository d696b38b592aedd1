set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7x
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r7x/tests_all.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/r7x/tests_all.log; exit 1; }
tail -1 gpurun_out/r7x/tests_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r7x/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r7x/smoke.log; exit 1; }
tail -2 gpurun_out/r7x/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r7x/bench.json 2> gpurun_out/r7x/bench.err || { echo "bench failed"; tail -20 gpurun_out/r7x/bench.err; exit 1; }
cat gpurun_out/r7x/bench.json
timeout -k 10 300 python -u scripts/glm_automl_prof.py > gpurun_out/r7x/glm_automl_prof.txt 2>&1 || { echo "glm prof failed"; tail -20 gpurun_out/r7x/glm_automl_prof.txt; exit 1; }
head -2 gpurun_out/r7x/glm_automl_prof.txt
