# Round-3 check: new GPU tests first (verbose), then the whole GPU suite and the default bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_distributed_gpu.py "tests/test_kmeans.py::test_lloyd_kernel_large_n_f64_accumulation" \
  "tests/test_deeplearning.py::test_dl_step_graph_matches_eager" -m gpu > gpurun_out/pytest_new.log 2>&1 || { echo "new tests failed"; tail -60 gpurun_out/pytest_new.log; exit 1; }
tail -n 6 gpurun_out/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-600
